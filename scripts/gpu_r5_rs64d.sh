#!/bin/bash
# Round 5: K = 64 with the block layout (no zero block; exp/libpml_glm_blk64.so) vs the packed triangle (production).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5rs64d
mkdir -p $out
PML_GLM_LIB=photon_ml_amd/ops/_lib/exp/libpml_glm_blk64.so timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "row_space_tron and 8" -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for lib in photon_ml_amd/ops/_lib/libpml_glm.so photon_ml_amd/ops/_lib/exp/libpml_glm_blk64.so; do
  t=$(basename $lib .so)
  PML_GLM_LIB=$lib timeout -k 10 300 python3 -u scripts/rs_tron_bench.py 200000 64 8,5 > $out/${t}.log 2>&1 || { echo "failed"; tail -20 $out/${t}.log; exit 1; }
  echo "== $t"; grep -v amdgpu.ids $out/${t}.log | grep -v ordered | tail -3
done
