#!/bin/bash
# Multi-chunk forward launch: kernel tests, in-process A/B (per-chunk vs one launch), rbits 9 vs 10, bench.py.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python __graft_entry__.py build > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/pytest_kernels.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_kernels.log; exit 1; }
tail -1 gpurun_out/pytest_kernels.log
timeout -k 10 600 python scripts/kbench.py --rows 16000000 --layout tiled --reps 7 --tl-configs "4,4,0,0;4,4,0,1;2,4,0,1;4,4,0,0;4,4,0,1;2,4,0,1" > gpurun_out/tl_multi_ab.log 2>&1 || { echo "kbench failed"; tail -30 gpurun_out/tl_multi_ab.log; exit 1; }
PML_TL_RBITS=9 timeout -k 10 600 python scripts/kbench.py --rows 16000000 --layout tiled --reps 7 --tl-configs "4,4,0,0;4,4,0,1;2,4,0,1;4,4,0,1" > gpurun_out/tl_multi_r9.log 2>&1 || { echo "kbench r9 failed"; tail -30 gpurun_out/tl_multi_r9.log; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/tl_multi_ab.log", "gpurun_out/tl_multi_r9.log"):
    print(f)
    for line in open(f):
        if line.startswith("{"):
            r = json.loads(line); print("  cfg %s: fwd %.3f t %.3f pass %.3f" % (r["cfg"], r["fwd_ms"], r["t_ms"], r["pass_ms"]))
PY
timeout -k 10 900 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_multi.json 2> gpurun_out/bench_multi.err || { echo "bench failed"; tail -20 gpurun_out/bench_multi.err; exit 1; }
cat gpurun_out/bench_multi.json
