#!/bin/bash
# Round 5 step 1: lean-kernel A/B (microbench), then the fast-path parity tests and the RE GPU tests.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5s1
mkdir -p $out
bash scripts/gpu_r5_lean_ab.sh old v3 v4a v4b v4c || exit 1
timeout -k 10 600 python -u -m pytest tests/test_fastpath_parity_gpu.py tests/test_game_gpu.py -x -v --timeout 200 --timeout-method thread -k "parity or fastpath or lean or fused or row_space or resident or overlap or router" > $out/pytest.log 2>&1 || { echo "pytest failed"; grep -E "PASS|FAIL|Error|error" $out/pytest.log | tail -30; tail -40 $out/pytest.log; exit 1; }
grep -cE "PASSED" $out/pytest.log; tail -3 $out/pytest.log
