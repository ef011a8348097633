#!/bin/bash
# Round 6 step 17: Frobenius norm at build time -- tests, fresh-process one-shot, cold + warm FE windows.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6s17
mkdir -p $out
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_game_gpu.py tests/test_fastpath_parity_gpu.py tests/test_lbfgs_plan_gpu.py > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 300 python -u scripts/oneshot_profile.py --precisions bf16,f64 --json $out/nosync.json > $out/nosync.md 2> $out/nosync.log || { echo "oneshot failed"; tail -30 $out/nosync.log; exit 1; }
grep -E "warm-up" $out/nosync.md
cd /tmp
PML_TRACE=1 timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace -d $out/prof -o prof -- python3 $R/scripts/oneshot_profile.py --precisions bf16 > $out/prof_run.md 2> $out/prof_run.log || { echo "prof failed"; tail -30 $out/prof_run.log; exit 1; }
db=$(find $out/prof -name "*.db" | head -1)
export PML_WIN_TIMELINE=0
PML_WIN_INDEX=0 python3 $R/scripts/prof_window.py "$db" "Update coordinate global" $out/win_cold_fe.md > /dev/null; sed -n 1,30p $out/win_cold_fe.md; grep -A10 "Idle gaps" $out/win_cold_fe.md
PML_WIN_INDEX=0 python3 $R/scripts/prof_window.py "$db" "Update coordinate per-entity" $out/win_cold_re.md > /dev/null; sed -n 1,12p $out/win_cold_re.md; grep -A8 "Idle gaps" $out/win_cold_re.md
rm -f $db
