#!/bin/bash
# Wide batched GEMV (row-space classes n > 64) numerics + the game5pl bench (materialisation inside the timed region).
set -o pipefail
mkdir -p gpurun_out/r4mat
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_game_gpu.py -x -q --timeout 200 --timeout-method thread -k "batched_small_gemv or row_space" > gpurun_out/r4mat/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r4mat/pytest.log; exit 1; }
tail -2 gpurun_out/r4mat/pytest.log
timeout -k 10 400 python -u bench_game.py --config game5pl --steps 5 --warmup 2 > gpurun_out/r4mat/game5pl.json 2> gpurun_out/r4mat/game5pl.log || { echo "game5pl failed"; tail -30 gpurun_out/r4mat/game5pl.log; exit 1; }
cut -c1-400 gpurun_out/r4mat/game5pl.json
grep "sweeps (ms)" gpurun_out/r4mat/game5pl.log
