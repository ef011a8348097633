#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python __graft_entry__.py build > gpurun_out/build.log 2>&1 || { echo "build failed"; exit 1; }
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py tests/test_game_gpu.py -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 900 python bench_game.py > gpurun_out/bench_game.json 2> gpurun_out/bench_game.log || { echo "bench failed"; tail -30 gpurun_out/bench_game.log; exit 1; }
cat gpurun_out/bench_game.json; tail -4 gpurun_out/bench_game.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_game -o prof -- python3 $GRAFT_REPO_ROOT/bench_game.py --entities-per-gpu 50000 --steps 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_game.log 2>&1 || { echo "prof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof_game.log; exit 1; }
cd $GRAFT_REPO_ROOT && python scripts/prof_summary.py $(find /tmp/prof_game -name "*.db" | head -1) gpurun_out/game_kernel_stats.md "bench_game.py --entities-per-gpu 50000 --steps 2" > /dev/null && head -22 gpurun_out/game_kernel_stats.md
