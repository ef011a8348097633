#!/bin/bash
# Bucketed / overlapped gradient all-reduce: bitwise tests, then 2 ranks on one GPU (gloo) with and without buckets.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "bucketed" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ov.log 2>&1 || { echo "pytest failed"; tail -50 gpurun_out/pytest_ov.log; exit 1; }
tail -1 gpurun_out/pytest_ov.log
for nb in 4 1; do
  PML_GRAD_BUCKETS=$nb PML_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2961$nb bench.py --gpus 2 --rows-per-gpu 8000000 --steps 3 --warmup 1 > gpurun_out/ov_$nb.json 2> gpurun_out/ov_$nb.log || { echo "2-rank nb=$nb failed"; tail -30 gpurun_out/ov_$nb.log; exit 1; }
  grep -h "final" gpurun_out/ov_$nb.log
done
timeout -k 10 300 python bench.py --rows-per-gpu 16000000 --steps 5 --warmup 2 > gpurun_out/ov_1gpu.json 2> gpurun_out/ov_1gpu.log || { echo "1gpu failed"; tail -30 gpurun_out/ov_1gpu.log; exit 1; }
grep -h final gpurun_out/ov_1gpu.log
