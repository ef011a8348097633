#!/bin/bash
# GAME on the GPU with the row-space random-effect solve: GAME GPU tests, config-5 bench (row space on / off).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_game_gpu.py tests/test_kernels_gpu.py -k "game or batched_small or segmented_random" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_game_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_game_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_game_gpu.log
timeout -k 10 900 python bench_game.py --config game5 --steps 3 --warmup 1 > gpurun_out/g5rs.json 2> gpurun_out/g5rs.log || { echo "game5 failed"; tail -30 gpurun_out/g5rs.log; exit 1; }
cat gpurun_out/g5rs.json
grep -v amdgpu.ids gpurun_out/g5rs.log | tail -6
