#!/bin/bash
# Round 6: whole GPU test tier + smoke + fresh-process one-shot phase table.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6full
mkdir -p $out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $out/pytest.log | tail -20; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
PML_SYNC_TIMED=1 timeout -k 10 300 python -u scripts/oneshot_profile.py --precisions bf16,f64 --json $out/phases.json > $out/phases.md 2> $out/phases.log || { echo "oneshot failed"; tail -30 $out/phases.log; exit 1; }
timeout -k 10 300 python -u scripts/oneshot_profile.py --precisions bf16,f64 --json $out/nosync.json > $out/nosync.md 2> $out/nosync.log || { echo "oneshot nosync failed"; tail -30 $out/nosync.log; exit 1; }
grep -E "warm-up" $out/phases.md $out/nosync.md
