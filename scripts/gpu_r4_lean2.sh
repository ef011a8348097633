#!/bin/bash
# Lean streaming RE kernel in production: GAME GPU tests, game5pl bench (bf16 + fp64 FE keys), RE / FE windows.
set -o pipefail
mkdir -p gpurun_out/r4lean3
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_game_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4lean3/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r4lean3/pytest.log; exit 1; }
tail -2 gpurun_out/r4lean3/pytest.log
timeout -k 10 400 python -u bench_game.py --config game5pl --steps 5 --warmup 2 > gpurun_out/r4lean3/game5pl.json 2> gpurun_out/r4lean3/game5pl.log || { echo "game5pl failed"; tail -30 gpurun_out/r4lean3/game5pl.log; exit 1; }
cut -c1-700 gpurun_out/r4lean3/game5pl.json
bash scripts/gpu_r4_window.sh game5pl g5pl_lean
