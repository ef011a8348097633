#!/bin/bash
# Fused row-space TRON kernel: parity tests vs the vectorised batched TRON, then the GAME config-5 bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_game_gpu.py -k "fused_row_space or batched_small or game or segmented_random" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_rs.log 2>&1 || { echo "pytest failed"; tail -50 gpurun_out/pytest_rs.log; exit 1; }
tail -1 gpurun_out/pytest_rs.log
rm -f gpurun_out/g5f_tl.jsonl
PML_TIMELINE=$GRAFT_REPO_ROOT/gpurun_out/g5f_tl.jsonl timeout -k 10 900 python bench_game.py --config game5 --steps 3 --warmup 1 > gpurun_out/g5f.json 2> gpurun_out/g5f.log || { echo "game5 failed"; tail -30 gpurun_out/g5f.log; exit 1; }
cat gpurun_out/g5f.json
grep -v amdgpu.ids gpurun_out/g5f.log | tail -8
