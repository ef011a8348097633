#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 500 python scripts/kbench.py --rows 8000000 --chunk-rows 1048576 --configs "0,0,0;0,1,0;0,0,8192;1,0,0" > gpurun_out/kbench2.jsonl 2> gpurun_out/kbench2.log || { tail -30 gpurun_out/kbench2.log; exit 1; }
cat gpurun_out/kbench2.jsonl
