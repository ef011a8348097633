#!/bin/bash
# Lane-interleaved TL layout: kernel parity tests, then in-process A/B (plain vs interleaved streams) on 16M rows.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_kern.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_kern.log; exit 1; }
tail -1 gpurun_out/pytest_kern.log
timeout -k 10 500 python scripts/kbench.py --rows 16000000 --chunk-rows 1048576 --il 0 1 --tl-configs "2,4,0,1,0;4,4,0,1,0;2,2,0,1,0" > gpurun_out/kbench_il.jsonl 2> gpurun_out/kbench_il.log || { tail -30 gpurun_out/kbench_il.log; exit 1; }
cat gpurun_out/kbench_il.jsonl
