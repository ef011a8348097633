#!/bin/bash
# New GAME kernels (scoring, MFMA Gram / GEMM) + CLI GPU tests, then the block/tile sweep.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_game_gpu.py tests/test_cli_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_game.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_game.log; exit 1; }
tail -2 gpurun_out/pytest_game.log
bash scripts/gpu_bits.sh
