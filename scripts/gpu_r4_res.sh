#!/bin/bash
# Round 4: register-resident fused primal TRON: fused GPU tests, the microbenchmark (stream vs resident), game5pl.
set -o pipefail
mkdir -p gpurun_out/r4res
export TMPDIR=/tmp
export PML_CHECK_KERNEL_INPUTS=1
timeout -k 10 600 python -u -m pytest tests/test_game_gpu.py -x -q --timeout 120 --timeout-method thread -k "fused" > gpurun_out/r4res/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r4res/pytest.log; exit 1; }
tail -1 gpurun_out/r4res/pytest.log
unset PML_CHECK_KERNEL_INPUTS
timeout -k 10 300 python -u scripts/re_fused_bench.py 43000 stream,res > gpurun_out/r4res/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r4res/bench.log; exit 1; }
cat gpurun_out/r4res/bench.log | grep -v amdgpu.ids
timeout -k 10 300 python -u scripts/fe_ops_profile.py game5pl gpurun_out/r4res/fe_ops.txt > gpurun_out/r4res/fe_ops.log 2>&1 || { echo "fe ops profile failed"; tail -20 gpurun_out/r4res/fe_ops.log; }
