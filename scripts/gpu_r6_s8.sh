#!/bin/bash
# Round 6 step 8: whole-iteration L-BFGS plans -- GPU tests, game5pl bench at both precisions, warm FE window.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6s8
mkdir -p $out
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_fastpath_parity_gpu.py tests/test_lbfgs_plan_gpu.py > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for p in bf16 f64; do
  timeout -k 10 300 python -u bench_game.py --config game5pl --steps 6 --warmup 3 --precision $p > $out/bench_$p.json 2> $out/bench_$p.log || { echo "bench $p failed"; tail -30 $out/bench_$p.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$out/bench_$p.json')); print('$p', {k: d.get(k) for k in ('ms_per_step','sweep_ms_median','coordinate_ms','cold_first_sweep_ms','fe_lbfgs_plans')})"
done
cd /tmp
PML_TRACE=1 timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace -d $out/prof -o prof -- python3 $R/scripts/oneshot_profile.py --precisions bf16 > $out/prof_run.md 2> $out/prof_run.log || { echo "prof failed"; tail -30 $out/prof_run.log; exit 1; }
db=$(find $out/prof -name "*.db" | head -1)
PML_WIN_INDEX=2 python3 $R/scripts/prof_window.py "$db" "Update coordinate global" $out/win_fe_warm.md > /dev/null; sed -n 1,30p $out/win_fe_warm.md; grep -A14 "Idle gaps" $out/win_fe_warm.md
rm -f $db
