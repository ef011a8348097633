#!/bin/bash
# GAME on the GPU: all gpu tests, GAME bench (small + default), profile of the GAME bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python __graft_entry__.py build > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 900 python -m pytest tests/ -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench_game.py --entities-per-gpu 20000 --rows-per-entity 50 --fe-dim 100000 > gpurun_out/bench_game_small.json 2> gpurun_out/bench_game_small.log || { echo "bench_game small failed"; tail -40 gpurun_out/bench_game_small.log; exit 1; }
cat gpurun_out/bench_game_small.json
timeout -k 10 900 python bench_game.py > gpurun_out/bench_game.json 2> gpurun_out/bench_game.log || { echo "bench_game failed"; tail -40 gpurun_out/bench_game.log; exit 1; }
cat gpurun_out/bench_game.json
tail -3 gpurun_out/bench_game.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_game -o prof -- python3 $GRAFT_REPO_ROOT/bench_game.py --entities-per-gpu 50000 --steps 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_game.log 2>&1 || { echo "prof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof_game.log; exit 1; }
echo prof ok
