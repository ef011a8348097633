#!/bin/bash
# Live-flag entity masks (no host syncs) + margin-cache scoring: tests, game5pl, and the L-BFGS Gram two-loop A/B
# on the GAME fixed effect and the headline bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_game_gpu.py tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -k "masked or segmented or row_space or cached_margins or bitwise or tiled" > gpurun_out/pytest_game6.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_game6.log; exit 1; }
tail -2 gpurun_out/pytest_game6.log
PML_SYNC_TIMING=1 PML_TRON_STATS=1 timeout -k 10 900 python -u bench_game.py --config game5pl --steps 3 --warmup 2 --log-level DEBUG > gpurun_out/bench_game5pl_v7.json 2> gpurun_out/bench_game5pl_v7.log || { echo "bench failed"; tail -30 gpurun_out/bench_game5pl_v7.log; exit 1; }
grep -E "entity-masked|block-diagonal TRON|coordinate (global|per-entity)" gpurun_out/bench_game5pl_v7.log | cut -c1-250 | tail -8
cat gpurun_out/bench_game5pl_v7.json
for g in default 262144; do
  if [ $g = default ]; then unset PML_LBFGS_GRAM_MIN_DIM; else export PML_LBFGS_GRAM_MIN_DIM=$g; fi
  timeout -k 10 900 python -u bench_game.py --config game5 --steps 3 --warmup 2 > gpurun_out/bench_game5_gram_$g.json 2> gpurun_out/bench_game5_gram_$g.log || { echo "game5 $g failed"; tail -30 gpurun_out/bench_game5_gram_$g.log; exit 1; }
  echo "game5 gram=$g"; grep -E "coordinate (global|per-entity)" gpurun_out/bench_game5_gram_$g.log | tail -2; cat gpurun_out/bench_game5_gram_$g.json | cut -c1-200
  timeout -k 10 900 python bench.py > gpurun_out/bench_gram_$g.json 2> gpurun_out/bench_gram_$g.log || { echo "bench $g failed"; tail -30 gpurun_out/bench_gram_$g.log; exit 1; }
  echo "bench gram=$g"; cat gpurun_out/bench_gram_$g.json | cut -c1-250
done
