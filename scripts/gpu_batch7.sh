#!/bin/bash
# GAME at BASELINE precision (fp64 fixed-effect features) next to bf16, the 2-rank entity-sharded rehearsal on one
# GPU, BASELINE configs 3/4, and the tall-narrow MFMA Hessian path.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in game5 game5pl; do
  timeout -k 10 600 python -u bench_game.py --config $cfg --steps 3 --warmup 2 --precision f64 > gpurun_out/${cfg}_f64.json 2> gpurun_out/${cfg}_f64.log || { echo "$cfg f64 failed"; tail -30 gpurun_out/${cfg}_f64.log; exit 1; }
  echo "$cfg f64:"; cut -c1-200 gpurun_out/${cfg}_f64.json; grep -o '"coordinate_ms".*' gpurun_out/${cfg}_f64.json
done
PML_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --rows-per-gpu 30000000 --steps 3 --warmup 1 > gpurun_out/bench_2rank_gloo_30M.json 2> gpurun_out/bench_2rank_gloo_30M.log || { echo "2-rank bench failed"; tail -30 gpurun_out/bench_2rank_gloo_30M.log; exit 1; }
cut -c1-400 gpurun_out/bench_2rank_gloo_30M.json
bash scripts/gpu_rehearsal.sh && bash scripts/gpu_cfg34.sh r3 && bash scripts/gpu_hess.sh
