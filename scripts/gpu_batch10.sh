#!/bin/bash
# Speculative next direction (L-BFGS): tests + headline; GAME at fp64 FE features; 2-rank gloo headline rehearsal.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_rccl_gpu.py tests/test_game_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_b10.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_b10.log; exit 1; }
tail -2 gpurun_out/pytest_b10.log
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --game off > gpurun_out/bench_b10.json 2> gpurun_out/bench_b10.log || { echo "bench failed"; tail -20 gpurun_out/bench_b10.log; exit 1; }
cut -c1-300 gpurun_out/bench_b10.json
for cfg in game5 game5pl; do
  timeout -k 10 600 python -u bench_game.py --config $cfg --steps 3 --warmup 2 --precision f64 > gpurun_out/${cfg}_f64.json 2> gpurun_out/${cfg}_f64.log || { echo "$cfg f64 failed"; tail -30 gpurun_out/${cfg}_f64.log; exit 1; }
  echo "$cfg f64:"; cut -c1-200 gpurun_out/${cfg}_f64.json; grep -o '"coordinate_ms".*' gpurun_out/${cfg}_f64.json
done
PML_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --rows-per-gpu 30000000 --steps 3 --warmup 1 --game off > gpurun_out/bench_2rank_gloo_30M.json 2> gpurun_out/bench_2rank_gloo_30M.log || { echo "2-rank bench failed"; tail -30 gpurun_out/bench_2rank_gloo_30M.log; exit 1; }
cut -c1-400 gpurun_out/bench_2rank_gloo_30M.json
