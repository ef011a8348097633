#!/bin/bash
# GAME config-5 shape, 2 ranks sharing one GPU over gloo (entity-sharded random effects + row-space solves)
# vs 1 rank with the same total entities: the training losses must agree.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
PML_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29631 bench_game.py --gpus 2 --config game5 --entities-per-gpu 100000 --steps 2 --warmup 1 > gpurun_out/g5_2rank.json 2> gpurun_out/g5_2rank.err || { echo "2rank failed"; grep -v amdgpu.ids gpurun_out/g5_2rank.err | tail -40; exit 1; }
grep -v amdgpu.ids gpurun_out/g5_2rank.err | grep "final training loss\|allocator" | cut -c1-200; cat gpurun_out/g5_2rank.json | cut -c1-200
