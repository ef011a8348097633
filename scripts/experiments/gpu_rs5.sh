#!/bin/bash
# rs_tron variant 5 (one wave per workgroup for the LDS-resident sizes) vs variant 3: correctness, then timings.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -k "fused_row_space_tron" > gpurun_out/pytest_rs5.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_rs5.log; exit 1; }
tail -2 gpurun_out/pytest_rs5.log
for n in 20 24 32; do
  timeout -k 10 300 python -u scripts/rs_tron_bench.py 1250000 $n 3,5 > gpurun_out/rs5_n$n.log 2>&1 || { echo "bench $n failed"; tail -30 gpurun_out/rs5_n$n.log; exit 1; }
  echo "n=$n"; cat gpurun_out/rs5_n$n.log
done
