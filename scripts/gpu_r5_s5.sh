#!/bin/bash
# Round 5 step 5: marginal-cost ablations of the lean kernel (extra atomic / gather / value load per entry, same
# iterates), the fast-path GPU tests, the headline PMC + bench, the counter list.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5s5
mkdir -p $out
rocprofv3 -L > $out/counters_list.txt 2>&1 || true
bash scripts/gpu_r5_lean_ab.sh s3 a1 a2 a4 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_fastpath_parity_gpu.py -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; grep -E "PASS|FAIL|Error|error" $out/pytest.log | tail -30; tail -40 $out/pytest.log; exit 1; }
grep -cE "PASSED" $out/pytest.log; tail -2 $out/pytest.log
bash scripts/gpu_r5_headpmc.sh
