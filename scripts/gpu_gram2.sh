#!/bin/bash
# Gram / lincomb kernels: tests, then A/B of the vector-free two-loop on the headline bench and GAME config 5.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "gram or vector_free" > gpurun_out/pytest_gram.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gram.log; exit 1; }
tail -1 gpurun_out/pytest_gram.log
bash scripts/gpu_gram.sh
