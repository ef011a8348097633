#!/bin/bash
# A/B of TL pipeline variants (kernel microbench) + bitwise tests of the deep variants.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "deep or narrow" > gpurun_out/pytest_deep.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_deep.log; exit 1; }
tail -2 gpurun_out/pytest_deep.log
timeout -k 10 500 python scripts/kbench.py --rows 16000000 --reps 5 --tl-configs "${AB_CONFIGS:-2,4,0,1,0,0,0,0;2,4,0,1,0,0,1,1;2,4,0,1,0,0,2,2;4,4,0,1,0,0,1,1;4,4,0,1,0,0,2,2}" > gpurun_out/kbench_ab.jsonl 2> gpurun_out/kbench_ab.log || { echo "kbench failed"; tail -30 gpurun_out/kbench_ab.log; exit 1; }
cat gpurun_out/kbench_ab.jsonl
