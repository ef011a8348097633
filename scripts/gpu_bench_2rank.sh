#!/bin/bash
# Rehearsal of the driver's multi-rank bench launch on the 1-GPU box: 2 ranks share the card over gloo
# (RCCL refuses two ranks on one device), reduced rows/GPU so both shards fit; then the GAME config-5 bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
PML_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 5 --warmup 2 --rows-per-gpu 16000000 \
  > gpurun_out/bench_2rank.json 2> gpurun_out/bench_2rank.log || { echo "2-rank bench failed"; tail -30 gpurun_out/bench_2rank.log; exit 1; }
cat gpurun_out/bench_2rank.json
timeout -k 10 500 python bench_game.py --config game5 --steps 5 > gpurun_out/bench_game.json 2> gpurun_out/bench_game.log || { echo "game bench failed"; tail -30 gpurun_out/bench_game.log; exit 1; }
cat gpurun_out/bench_game.json
