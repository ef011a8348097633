#!/bin/bash
# Iteration run: TL kernel GPU tests, then the headline bench at a reduced row count and at full size.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_kernels.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_kernels.log; exit 1; }
tail -3 gpurun_out/pytest_kernels.log
timeout -k 10 600 python bench.py --rows-per-gpu 32000000 --steps 10 --warmup 3 > gpurun_out/bench_32M.json 2> gpurun_out/bench_32M.log || { echo "bench 32M failed"; tail -40 gpurun_out/bench_32M.log; exit 1; }
cat gpurun_out/bench_32M.json
timeout -k 10 900 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.log || { echo "full bench failed"; tail -40 gpurun_out/bench_full.log; exit 1; }
cat gpurun_out/bench_full.json
