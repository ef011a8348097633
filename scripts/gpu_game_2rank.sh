#!/bin/bash
# 2-rank GAME rehearsal on one GPU: both ranks share the device, so collectives use gloo (RCCL refuses two ranks
# on one GPU); the entity sharding / row routing / distributed evaluation paths are the production ones.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python __graft_entry__.py build > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
PML_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench_game.py --gpus 2 --config game5 --entities-per-gpu 100000 --steps 2 --warmup 1 > gpurun_out/bench_game5_2rank.json 2> gpurun_out/bench_game5_2rank.err || { echo "2rank failed"; grep -v amdgpu.ids gpurun_out/bench_game5_2rank.err | grep -A3 Error | head -40; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_game5_2rank.err | grep bench_game | tail -4; cat gpurun_out/bench_game5_2rank.json
timeout -k 10 600 python bench_game.py --config game5 --entities-per-gpu 200000 --steps 2 --warmup 1 > gpurun_out/bench_game5_1rank.json 2> gpurun_out/bench_game5_1rank.err || { echo "1rank failed"; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_game5_1rank.err | grep bench_game | tail -4
