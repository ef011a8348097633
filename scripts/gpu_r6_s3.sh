#!/bin/bash
# Round 6 step 3: row-space setup kernels (staged Gram, batched Cholesky) + one-shot phases + HIP API trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6s3
mkdir -p $out
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_game_gpu.py tests/test_kernels_gpu.py -k "gram or cholesky or row_space or key_hist" > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
PML_SYNC_TIMED=1 timeout -k 10 300 python -u scripts/oneshot_profile.py --precisions bf16,f64 --json $out/phases.json > $out/phases.md 2> $out/phases.log || { echo "oneshot failed"; tail -30 $out/phases.log; exit 1; }
cat $out/phases.md
cd /tmp
PML_TRACE=1 timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --hip-runtime-trace -d $out/prof -o prof -- python3 $R/scripts/oneshot_profile.py --precisions bf16 > $out/api_run.md 2> $out/api_run.log || { echo "prof failed"; tail -30 $out/api_run.log; exit 1; }
head -4 $out/api_run.md
db=$(find $out/prof -name "*.db" | head -1)
for w in "Update coordinate global" "Update coordinate per-entity"; do
  f=$out/api_$(echo "$w" | tr -c 'a-zA-Z0-9' '_').md
  python3 $R/scripts/prof_api_window.py "$db" "$w" 0 > $f && head -30 $f
done
export PML_WIN_TIMELINE=0
PML_WIN_INDEX=0 python3 $R/scripts/prof_window.py "$db" "Update coordinate global" $out/win_cold_fe.md > /dev/null && sed -n 1,12p $out/win_cold_fe.md && grep -A12 "Idle gaps" $out/win_cold_fe.md
PML_WIN_INDEX=0 python3 $R/scripts/prof_window.py "$db" "Update coordinate per-entity" $out/win_cold_re.md > /dev/null && sed -n 1,30p $out/win_cold_re.md
rm -f $db
