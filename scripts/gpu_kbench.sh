#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 400 python scripts/kbench.py --rows 8000000 --chunk-rows 262144 524288 1048576 2097152 > gpurun_out/kbench.jsonl 2> gpurun_out/kbench.log || { tail -30 gpurun_out/kbench.log; exit 1; }
cat gpurun_out/kbench.jsonl
