#!/bin/bash
# 8-entries-per-lane stream variant: kernel tests + in-process A/B (fwd/T pipe 0 vs 2).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python __graft_entry__.py build > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/pytest_kernels.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_kernels.log; exit 1; }
tail -1 gpurun_out/pytest_kernels.log
# cfg: waves, waves_t, pipe_fwd, multi, pipe_t
timeout -k 10 600 python scripts/kbench.py --rows 16000000 --layout tiled --reps 7 --tl-configs "2,4,0,1,0;2,4,2,1,2;4,4,2,1,2;2,2,2,1,2;2,4,0,1,0;2,4,2,1,2;4,4,2,1,2;2,2,2,1,2" > gpurun_out/tl_wide.log 2>&1 || { echo "kbench failed"; tail -30 gpurun_out/tl_wide.log; exit 1; }
python3 - <<'PY'
import json
for line in open("gpurun_out/tl_wide.log"):
    if line.startswith("{"):
        r = json.loads(line); print("cfg %s: fwd %.3f t %.3f pass %.3f" % (r["cfg"], r["fwd_ms"], r["t_ms"], r["pass_ms"]))
PY
