#!/bin/bash
# Round 5: row-space TRON for n in (32, 64]: one problem per wave with permlane block rotation + DPP broadcast FMAs
# (variant 8) vs rs_tron_kernel<2> (variant 5 for n > 32). Tests, then the micro at 200K problems.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5rs64
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "rs_tron or row_space_tron" -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" $out/pytest.log | tail -30; tail -40 $out/pytest.log; exit 1; }
grep -cE "PASSED" $out/pytest.log; tail -1 $out/pytest.log
for n in ${NS:-40 48 64}; do
  timeout -k 10 300 python3 -u scripts/rs_tron_bench.py 200000 $n 5,8 > $out/rs_n$n.log 2>&1 || { echo "n=$n failed"; tail -20 $out/rs_n$n.log; exit 1; }
  echo "== n=$n"; grep -v amdgpu.ids $out/rs_n$n.log | grep -v ordered
done
