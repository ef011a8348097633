#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python __graft_entry__.py build > gpurun_out/build.log 2>&1 || { echo "build failed"; exit 1; }
timeout -k 10 600 python -m pytest tests/test_game_gpu.py -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 900 python bench_game.py > gpurun_out/bench_game.json 2> gpurun_out/bench_game.log || { echo "bench failed"; tail -30 gpurun_out/bench_game.log; exit 1; }
cat gpurun_out/bench_game.json; tail -4 gpurun_out/bench_game.log
timeout -k 10 900 python -m cProfile -o gpurun_out/game.pstats bench_game.py --steps 1 > /dev/null 2> gpurun_out/bench_game_cprof.log || { echo "cprofile failed"; tail -30 gpurun_out/bench_game_cprof.log; exit 1; }
python -c "import pstats; pstats.Stats('gpurun_out/game.pstats').sort_stats('cumulative').print_stats(45)" > gpurun_out/game_pstats.txt
