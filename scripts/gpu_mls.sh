#!/bin/bash
# Margin-space line search: device tests, full GPU tier, headline bench, 2-rank rehearsal, GAME config 5.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 900 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.log || { echo "bench failed"; tail -30 gpurun_out/bench_full.log; exit 1; }
cat gpurun_out/bench_full.json; grep -h final gpurun_out/bench_full.log
PML_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29617 bench.py --gpus 2 --rows-per-gpu 8000000 --steps 3 --warmup 1 > gpurun_out/mls2.json 2> gpurun_out/mls2.log || { echo "2-rank failed"; tail -30 gpurun_out/mls2.log; exit 1; }
grep -h "final\|all-reduce" gpurun_out/mls2.log
