#!/bin/bash
# Round 6: histogram kernel test + one-shot phase table + host profile of the one-shot run (no device syncs).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6oneshot2
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "key_histogram or tl_multi or column_windows or narrow or empty" > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
PML_SYNC_TIMED=1 timeout -k 10 300 python -u scripts/oneshot_profile.py --precisions bf16,f64 --json $out/phases.json > $out/phases.md 2> $out/phases.log || { echo "oneshot failed"; tail -30 $out/phases.log; exit 1; }
cat $out/phases.md
timeout -k 10 300 python -u scripts/oneshot_profile.py --precisions bf16,f64 --json $out/nosync.json --cprofile $out/cprofile_tottime.txt --cprofile-sort tottime > $out/nosync.md 2> $out/nosync.log || { echo "oneshot nosync failed"; tail -30 $out/nosync.log; exit 1; }
grep -E "coordinate build" $out/nosync.md
