#!/bin/bash
# Round 5 step 2: strided-row-pass lean variants (uniform TRON scalars), then the fast-path / RE GPU tests, the
# FE torch-call attribution and the fp64-vs-bf16 FE PMC.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5s2
mkdir -p $out
bash scripts/gpu_r5_lean_ab.sh s3 s4a s4b s3h4 s3f1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_fastpath_parity_gpu.py tests/test_game_gpu.py -x -v --timeout 200 --timeout-method thread -k "parity or fastpath or lean or fused or row_space or resident or overlap or router" > $out/pytest.log 2>&1 || { echo "pytest failed"; grep -E "PASS|FAIL|Error|error" $out/pytest.log | tail -30; tail -40 $out/pytest.log; exit 1; }
grep -cE "PASSED" $out/pytest.log; tail -3 $out/pytest.log
timeout -k 10 400 python -u scripts/fe_torch_calls.py game5pl $out/fe_torch_calls.txt > $out/fe_torch_calls.log 2>&1 || { echo "torch calls failed"; tail -20 $out/fe_torch_calls.log; exit 1; }
head -60 $out/fe_torch_calls.txt
bash scripts/gpu_r5_fepmc.sh
