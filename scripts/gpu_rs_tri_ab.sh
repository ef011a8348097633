#!/bin/bash
# Packed-triangular LDS layout of the general row-space TRON kernel (variant 2, classes n > 32): parity tests of
# every variant, then new vs previous library (abtmp/libpml_glm_old.so, built from the parent commit) on the
# n = 48 / 64 microbenchmark, alternating.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "fused_row_space_tron or rs_tron" --timeout 150 --timeout-method thread > gpurun_out/pytest_rstri.log 2>&1 || { tail -n 30 gpurun_out/pytest_rstri.log; exit 1; }
tail -n 1 gpurun_out/pytest_rstri.log
cp photon_ml_amd/ops/_lib/libpml_glm.so abtmp/libpml_glm_new.so
for lib in new old new old; do
  cp abtmp/libpml_glm_$lib.so photon_ml_amd/ops/_lib/libpml_glm.so
  for n in 48 64; do
    timeout -k 10 120 python scripts/rs_tron_bench.py 60000 $n 2 > gpurun_out/rs_${lib}_$n.log 2>&1 || { tail -n 20 gpurun_out/rs_${lib}_$n.log; exit 1; }
    echo "$lib n=$n: $(grep 'variant 2:' gpurun_out/rs_${lib}_$n.log | tail -n 1)"
  done
done
cp abtmp/libpml_glm_new.so photon_ml_amd/ops/_lib/libpml_glm.so
