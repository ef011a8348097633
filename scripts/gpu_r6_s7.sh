#!/bin/bash
# Round 6: remaining GPU tests (parity suite onwards) + CLI one-shot at scale (Avro -> game-training -> saved model).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6s7
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_re_parity_gpu.py tests/test_rccl_gpu.py tests/test_sanitizers.py tests/test_tiled_layout.py tests/test_watchdog.py -m gpu > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
PML_SYNC_TIMED=1 timeout -k 10 900 python -u scripts/cli_oneshot.py --records 10000000 --nnz 30 --entities 500000 --dir /tmp/pml_cli --out $out/cli.json > $out/cli.log 2>&1 || { echo "cli failed"; tail -30 $out/cli.log; exit 1; }
cat $out/cli.json
timeout -k 10 600 python -u scripts/oneshot_profile.py --precisions bf16,f64 --json $out/oneshot_nosync.json > $out/oneshot_nosync.md 2>&1 || { echo "oneshot failed"; tail -30 $out/oneshot_nosync.md; exit 1; }
grep -E "^runtime warm-up" $out/oneshot_nosync.md
