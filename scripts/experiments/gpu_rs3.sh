#!/bin/bash
# rs_tron variant 3 (DPP64 broadcasts): correctness vs batched TRON, then the 1.25M x 20 microbench + sizes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -k "fused_row_space_tron" > gpurun_out/pytest_rs3.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_rs3.log; exit 1; }
tail -2 gpurun_out/pytest_rs3.log
timeout -k 10 300 python -u scripts/rs_tron_bench.py 1250000 20 2,3,4 > gpurun_out/rs3_n20.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/rs3_n20.log; exit 1; }
cat gpurun_out/rs3_n20.log
for n in 8 12 16 24 32; do
  timeout -k 10 300 python -u scripts/rs_tron_bench.py 1250000 $n 2,3,4 > gpurun_out/rs3_n$n.log 2>&1 || { echo "bench $n failed"; tail -30 gpurun_out/rs3_n$n.log; exit 1; }
  echo "n=$n"; cat gpurun_out/rs3_n$n.log
done
