#!/bin/bash
# GPU validation: kernel parity tests, smoke, small + full bench. Each GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -40 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --rows-per-gpu 8000000 --steps 5 --warmup 2 > gpurun_out/bench_small.json 2> gpurun_out/bench_small.log || { echo "small bench failed"; tail -40 gpurun_out/bench_small.log; exit 1; }
cat gpurun_out/bench_small.json
timeout -k 10 900 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.log || { echo "full bench failed"; tail -40 gpurun_out/bench_full.log; exit 1; }
cat gpurun_out/bench_full.json
tail -5 gpurun_out/bench_full.log
