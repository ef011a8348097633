#!/bin/bash
# Lazy zero-point gradient tolerance + deferred loss read: tests, headline, game5 / game5pl, game5 FE window.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_game_gpu.py tests/test_downsample_gpu.py tests/test_sampling.py tests/test_rccl_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_b9.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_b9.log; exit 1; }
tail -2 gpurun_out/pytest_b9.log
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_b9.json 2> gpurun_out/bench_b9.log || { echo "bench failed"; tail -20 gpurun_out/bench_b9.log; exit 1; }
cut -c1-300 gpurun_out/bench_b9.json; grep -o '"game5pl_[a-z_]*": [0-9.]*' gpurun_out/bench_b9.json
timeout -k 10 600 python -u bench_game.py --config game5 --steps 3 --warmup 2 > gpurun_out/game5_b9.json 2> gpurun_out/game5_b9.log || { echo "game5 failed"; tail -30 gpurun_out/game5_b9.log; exit 1; }
cut -c1-200 gpurun_out/game5_b9.json; grep -o '"coordinate_ms".*' gpurun_out/game5_b9.json
cd /tmp
PML_TRACE=1 timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace -d $R/gpurun_out/prof_g5 -o prof -- python3 $R/bench_game.py --config game5 --steps 1 --warmup 2 > $R/gpurun_out/gaps_g5.json 2> $R/gpurun_out/gaps_g5.log || { echo "game prof failed"; tail -30 $R/gpurun_out/gaps_g5.log; exit 1; }
db=$(find $R/gpurun_out/prof_g5 -name "*.db" | head -1)
python3 $R/scripts/prof_window.py "$db" "Update coordinate global" $R/gpurun_out/game5_fe_window_b9.md > /dev/null && head -12 $R/gpurun_out/game5_fe_window_b9.md
rm -rf $R/gpurun_out/prof_g5
