#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python __graft_entry__.py build > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/pytest_kernels.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_kernels.log; exit 1; }
tail -1 gpurun_out/pytest_kernels.log
PML_TL_PIPE=1 timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -k "tiled" > gpurun_out/pytest_kernels_p1.log 2>&1 || { echo "pytest p1 failed"; tail -40 gpurun_out/pytest_kernels_p1.log; exit 1; }
tail -1 gpurun_out/pytest_kernels_p1.log
timeout -k 10 600 python scripts/kbench.py --rows 16000000 --layout tiled --reps 7 --tl-configs "4,4,0;4,4,1;2,2,0;2,2,1;4,4,0;4,4,1" > gpurun_out/tl_ab.log 2>&1 || { echo "kbench failed"; tail -30 gpurun_out/tl_ab.log; exit 1; }
python3 - <<'PY'
import json
for line in open("gpurun_out/tl_ab.log"):
    if line.startswith("{"):
        r = json.loads(line); print("cfg %s: fwd %.3f t %.3f pass %.3f" % (r["cfg"], r["fwd_ms"], r["t_ms"], r["pass_ms"]))
PY
