#!/bin/bash
# Fused per-entity primal TRON: GPU tests, then the power-law GAME bench with per-phase timings.
# Usage: bash scripts/gpu_fused.sh <tag>
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-fused}
timeout -k 10 600 python -u -m pytest tests/test_game_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_$tag.log; exit 1; }
tail -3 gpurun_out/pytest_$tag.log
PML_SYNC_TIMING=1 timeout -k 10 900 python -u bench_game.py --config game5pl --steps 3 --warmup 2 --log-level DEBUG > gpurun_out/game5pl_$tag.json 2> gpurun_out/game5pl_$tag.log || { echo "game5pl failed"; tail -40 gpurun_out/game5pl_$tag.log; exit 1; }
grep -E "RE per-entity|coordinate (global|per-entity)|entities" gpurun_out/game5pl_$tag.log | tail -24
cut -c1-300 gpurun_out/game5pl_$tag.json
