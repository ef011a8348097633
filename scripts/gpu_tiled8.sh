#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python __graft_entry__.py build > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/pytest_kernels.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_kernels.log; exit 1; }
tail -1 gpurun_out/pytest_kernels.log
timeout -k 10 300 python scripts/kbench.py --rows 16000000 --layout tiled --configs "0,0,0" > gpurun_out/kbp2.log 2>&1 || { echo "kbench failed"; tail -30 gpurun_out/kbp2.log; exit 1; }
tail -1 gpurun_out/kbp2.log
# distributed bench flow: 2 ranks sharing the one GPU over gloo (RCCL needs one GPU per rank)
PML_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --rows-per-gpu 4000000 --steps 3 --warmup 1 > gpurun_out/bench_2rank.json 2> gpurun_out/bench_2rank.log || { echo "2-rank bench failed"; tail -40 gpurun_out/bench_2rank.log; exit 1; }
cat gpurun_out/bench_2rank.json
PML_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29556 bench_game.py --gpus 2 --entities-per-gpu 20000 --fe-dim 100000 --steps 2 > gpurun_out/bench_game_2rank.json 2> gpurun_out/bench_game_2rank.log || { echo "2-rank game bench failed"; tail -40 gpurun_out/bench_game_2rank.log; exit 1; }
cat gpurun_out/bench_game_2rank.json
