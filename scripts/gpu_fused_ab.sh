#!/bin/bash
# Fused primal TRON row-pass A/B on game5pl (+ the GAME GPU tests first).
# Usage: bash scripts/gpu_fused_ab.sh <tag> [variants...]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-ab}; shift
vars=${@:-"2 1"}
timeout -k 10 600 python -u -m pytest tests/test_game_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_$tag.log; exit 1; }
tail -2 gpurun_out/pytest_$tag.log
for v in $vars; do
  PML_RE_ROWPASS=$v PML_SYNC_TIMING=1 timeout -k 10 600 python -u bench_game.py --config game5pl --steps 3 --warmup 2 --log-level DEBUG > gpurun_out/game5pl_${tag}_v$v.json 2> gpurun_out/game5pl_${tag}_v$v.log || { echo "game5pl v$v failed"; tail -40 gpurun_out/game5pl_${tag}_v$v.log; exit 1; }
  echo "variant $v:"; grep -E "fused primal solve|row-space solve" gpurun_out/game5pl_${tag}_v$v.log | tail -2
  cut -c1-220 gpurun_out/game5pl_${tag}_v$v.json
done
