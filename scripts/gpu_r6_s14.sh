#!/bin/bash
# Round 6 step 14: gated first-trial finish -- tests, A/B on game5pl (bf16 x2, fp64), warm FE window.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6s14
mkdir -p $out
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_lbfgs_plan_gpu.py tests/test_fastpath_parity_gpu.py tests/test_kernels_gpu.py > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for cfg in "0 bf16 a" "1 bf16 a" "0 bf16 b" "1 bf16 b" "0 f64 a" "1 f64 a"; do
  set -- $cfg
  PML_LBFGS_GATED=$1 timeout -k 10 300 python -u bench_game.py --config game5pl --steps 10 --warmup 3 --precision $2 > $out/bench_g$1_$2_$3.json 2> $out/bench_g$1_$2_$3.log || { echo "bench $cfg failed"; tail -30 $out/bench_g$1_$2_$3.log; exit 1; }
  python3 -c "import json; d=json.load(open('$out/bench_g$1_$2_$3.json')); print('gated $1 $2 $3', round(d['ms_per_step'],2), round(d['sweep_ms_median'],2), {k: round(v,2) for k,v in d['coordinate_ms'].items()})"
done
cd /tmp
PML_TRACE=1 timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace -d $out/prof -o prof -- python3 $R/scripts/oneshot_profile.py --precisions bf16 > $out/prof_run.md 2> $out/prof_run.log || { echo "prof failed"; tail -30 $out/prof_run.log; exit 1; }
db=$(find $out/prof -name "*.db" | head -1)
PML_WIN_INDEX=-1 python3 $R/scripts/prof_window.py "$db" "Update coordinate global" $out/win_fe_warm.md > /dev/null; sed -n 1,30p $out/win_fe_warm.md; grep -A12 "Idle gaps" $out/win_fe_warm.md
rm -f $db
