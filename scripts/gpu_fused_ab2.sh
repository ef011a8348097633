#!/bin/bash
# Fused primal TRON: GAME GPU tests, kernel microbench, game5pl with row-space nmax 64 vs 32.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-ab2}
timeout -k 10 600 python -u -m pytest tests/test_game_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_$tag.log; exit 1; }
tail -2 gpurun_out/pytest_$tag.log
timeout -k 10 300 python -u scripts/re_fused_bench.py 43000 2 > gpurun_out/re_fused_bench_$tag.log 2>&1 || { echo "microbench failed"; tail -20 gpurun_out/re_fused_bench_$tag.log; exit 1; }
cat gpurun_out/re_fused_bench_$tag.log
for nm in 64 32; do
  PML_RS_NMAX=$nm PML_SYNC_TIMING=1 timeout -k 10 600 python -u bench_game.py --config game5pl --steps 3 --warmup 2 --log-level DEBUG > gpurun_out/game5pl_${tag}_nm$nm.json 2> gpurun_out/game5pl_${tag}_nm$nm.log || { echo "game5pl nm$nm failed"; tail -40 gpurun_out/game5pl_${tag}_nm$nm.log; exit 1; }
  echo "nmax $nm:"; grep -E "fused primal solve|row-space solve|fused primal, " gpurun_out/game5pl_${tag}_nm$nm.log | tail -3
  cut -c1-220 gpurun_out/game5pl_${tag}_nm$nm.json
done
