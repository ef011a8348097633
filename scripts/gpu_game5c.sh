#!/bin/bash
# seg_expand + dzz cache: kernel tests, config-5 bench (1 GPU), 2-rank GAME rehearsal on one GPU (nccl).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python __graft_entry__.py build > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_game_gpu.py -x -q > gpurun_out/pytest_k.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_k.log; exit 1; }
tail -1 gpurun_out/pytest_k.log
timeout -k 10 1000 python bench_game.py --config game5 --steps 2 --warmup 1 > gpurun_out/bench_game5.json 2> gpurun_out/bench_game5.err || { echo "game5 failed"; tail -20 gpurun_out/bench_game5.err; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_game5.err | tail -3; cat gpurun_out/bench_game5.json
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench_game.py --gpus 2 --config game5 --entities-per-gpu 100000 --steps 2 --warmup 1 > gpurun_out/bench_game5_2rank.json 2> gpurun_out/bench_game5_2rank.err || { echo "2rank failed"; tail -30 gpurun_out/bench_game5_2rank.err; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_game5_2rank.err | grep bench_game | tail -4; cat gpurun_out/bench_game5_2rank.json
