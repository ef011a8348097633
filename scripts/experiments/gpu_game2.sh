#!/bin/bash
# GAME power-law preset after the primal entity-subset change, + device two-loop test + headline bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_game_gpu.py tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -k "two_loop or random_effect or segmented or row_space or game" > gpurun_out/pytest_game3.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_game3.log; exit 1; }
tail -2 gpurun_out/pytest_game3.log
timeout -k 10 900 python -u bench_game.py --config game5pl --steps 3 --warmup 3 > gpurun_out/bench_game5pl.json 2> gpurun_out/bench_game5pl.log || { echo "bench failed"; tail -30 gpurun_out/bench_game5pl.log; exit 1; }
grep -E "built in|iteration|final" gpurun_out/bench_game5pl.log | tail -8
cat gpurun_out/bench_game5pl.json
timeout -k 10 900 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.log || { echo "full bench failed"; tail -40 gpurun_out/bench_full.log; exit 1; }
cat gpurun_out/bench_full.json
