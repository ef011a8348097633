#!/bin/bash
# Round 5: variant 8 layout A/B for n in (32, 64]: 16 x 16 lower blocks + one zero block (production) vs the masked
# packed triangle (exp/libpml_glm_blk0.so).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5rs64c
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "rs_tron or row_space_tron" -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for n in 40 48 64; do
  for lib in photon_ml_amd/ops/_lib/libpml_glm.so photon_ml_amd/ops/_lib/exp/libpml_glm_blk0.so; do
    t=$(basename $lib .so)
    PML_GLM_LIB=$lib timeout -k 10 300 python3 -u scripts/rs_tron_bench.py 200000 $n 8,5 > $out/${t}_n$n.log 2>&1 || { echo "n=$n failed"; tail -20 $out/${t}_n$n.log; exit 1; }
    echo "== $t n=$n"; grep -v amdgpu.ids $out/${t}_n$n.log | grep -v ordered | tail -3
  done
done
