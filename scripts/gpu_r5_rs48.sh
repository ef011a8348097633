#!/bin/bash
# Round 5: K = 48 block layout without the zero block (above-diagonal terms take a zero vector block): rs tests, micro.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5rs48
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "rs_tron or row_space_tron" -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for n in 40 48; do
  timeout -k 10 300 python3 -u scripts/rs_tron_bench.py 200000 $n 8,5 > $out/n$n.log 2>&1 || { echo "n=$n failed"; tail -20 $out/n$n.log; exit 1; }
  echo "== n=$n"; grep -v amdgpu.ids $out/n$n.log | grep -v ordered | tail -3
done
