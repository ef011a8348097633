#!/bin/bash
# Row-sampled fixed-effect updates (narrow sharing / filtering, derived launch tables, inherited margins), cheaper
# logistic loss math + wider ls_eval grid, zero-weight rows exact: tests, headline, and game5 down-sampling on
# click-like labels (~5 % positives) at rate 1.0 / 0.1, plus the FE window.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_downsample_gpu.py tests/test_sampling.py tests/test_kernels_gpu.py tests/test_game_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_b8.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_b8.log; exit 1; }
tail -2 gpurun_out/pytest_b8.log
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --game off > gpurun_out/bench_b8.json 2> gpurun_out/bench_b8.log || { echo "bench failed"; tail -20 gpurun_out/bench_b8.log; exit 1; }
cut -c1-300 gpurun_out/bench_b8.json
for r in 1.0 0.1; do
  timeout -k 10 600 python -u bench_game.py --config game5 --steps 3 --warmup 2 --label-bias -4 --fe-down-sampling-rate $r > gpurun_out/game5_ctr_ds$r.json 2> gpurun_out/game5_ctr_ds$r.log || { echo "game5 ds $r failed"; tail -30 gpurun_out/game5_ctr_ds$r.log; exit 1; }
  echo "rate $r:"; cut -c1-200 gpurun_out/game5_ctr_ds$r.json; grep -o '"label_bias".*' gpurun_out/game5_ctr_ds$r.json | cut -c1-400
done
cd /tmp
PML_TRACE=1 timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace -d $R/gpurun_out/prof_g5 -o prof -- python3 $R/bench_game.py --config game5 --steps 1 --warmup 2 > $R/gpurun_out/gaps_g5.json 2> $R/gpurun_out/gaps_g5.log || { echo "game prof failed"; tail -30 $R/gpurun_out/gaps_g5.log; exit 1; }
db=$(find $R/gpurun_out/prof_g5 -name "*.db" | head -1)
python3 $R/scripts/prof_window.py "$db" "Update coordinate global" $R/gpurun_out/game5_fe_window_b8.md > /dev/null && head -24 $R/gpurun_out/game5_fe_window_b8.md
rm -rf $R/gpurun_out/prof_g5
