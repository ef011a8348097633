#!/bin/bash
# Round 5 step 4: pipelined Hessian-vector pass A/B (lean kernel), fast-path GPU tests, headline PMC + floor.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5s4
mkdir -p $out
bash scripts/gpu_r5_lean_ab.sh s3 p2 p3 p2f1 s3 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_fastpath_parity_gpu.py -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; grep -E "PASS|FAIL|Error|error" $out/pytest.log | tail -30; tail -40 $out/pytest.log; exit 1; }
grep -cE "PASSED" $out/pytest.log; tail -2 $out/pytest.log
bash scripts/gpu_r5_headpmc.sh
