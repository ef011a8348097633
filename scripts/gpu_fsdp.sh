#!/bin/bash
# Feature-sharded optimizer state on the GPU: 1 rank (RCCL-free) and 2 ranks sharing the GPU over gloo.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python scripts/gram_bench.py && timeout -k 10 300 python bench.py --rows-per-gpu 16000000 --steps 5 --warmup 2 --optimizer-state feature-sharded > gpurun_out/fs1.json 2> gpurun_out/fs1.log || { echo "fs1 failed"; tail -30 gpurun_out/fs1.log; exit 1; }
cat gpurun_out/fs1.json
timeout -k 10 300 python bench.py --rows-per-gpu 16000000 --steps 5 --warmup 2 > gpurun_out/rep1.json 2> gpurun_out/rep1.log || { echo "rep1 failed"; tail -30 gpurun_out/rep1.log; exit 1; }
cat gpurun_out/rep1.json
PML_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --rows-per-gpu 8000000 --steps 3 --warmup 1 --optimizer-state feature-sharded > gpurun_out/fs2.json 2> gpurun_out/fs2.log || { echo "fs2 failed"; tail -30 gpurun_out/fs2.log; exit 1; }
cat gpurun_out/fs2.json
