#!/bin/bash
# Shard-wide transpose: kernel tests, in-process A/B (per-chunk vs one launch), chunk sizes, bench.py, profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python __graft_entry__.py build > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/pytest_kernels.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_kernels.log; exit 1; }
tail -1 gpurun_out/pytest_kernels.log
timeout -k 10 600 python scripts/kbench.py --rows 16000000 --layout tiled --reps 7 --chunk-rows 1048576 4194304 --tl-configs "2,4,0,0;2,4,0,1;2,2,0,1;2,4,0,0;2,4,0,1;2,2,0,1" > gpurun_out/tl_multi2.log 2>&1 || { echo "kbench failed"; tail -30 gpurun_out/tl_multi2.log; exit 1; }
python3 - <<'PY'
import json
for line in open("gpurun_out/tl_multi2.log"):
    if line.startswith("{"):
        r = json.loads(line); print("chunk %d cfg %s: fwd %.3f t %.3f pass %.3f" % (r["chunk_rows"], r["cfg"], r["fwd_ms"], r["t_ms"], r["pass_ms"]))
PY
timeout -k 10 900 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_multi2.json 2> gpurun_out/bench_multi2.err || { echo "bench failed"; tail -20 gpurun_out/bench_multi2.err; exit 1; }
cat gpurun_out/bench_multi2.json
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_kb -o prof -- python3 $GRAFT_REPO_ROOT/scripts/kbench.py --rows 16000000 --layout tiled --reps 5 --tl-configs "2,4,0,1" > $GRAFT_REPO_ROOT/gpurun_out/prof_kb.log 2>&1 || { echo "prof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof_kb.log; exit 1; }
cd $GRAFT_REPO_ROOT && python scripts/prof_summary.py $(find /tmp/prof_kb -name "*.db" | head -1) gpurun_out/kb_kernel_stats.md "kbench 16M rows tiled, 1M-row chunks, shard-wide launches" > /dev/null && cat gpurun_out/kb_kernel_stats.md
