#!/bin/bash
# Chunk-size A/B for the tiled transpose (launch count vs item size) + kernel profile of kbench at 1M-row chunks.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python __graft_entry__.py build > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python scripts/kbench.py --rows 16000000 --layout tiled --reps 7 --chunk-rows 1048576 2097152 4194304 --tl-configs "2,4,0,1" > gpurun_out/tl_chunks.log 2>&1 || { echo "kbench failed"; tail -30 gpurun_out/tl_chunks.log; exit 1; }
python3 - <<'PY'
import json
for line in open("gpurun_out/tl_chunks.log"):
    if line.startswith("{"):
        r = json.loads(line); print("chunk %d cfg %s: fwd %.3f t %.3f pass %.3f" % (r["chunk_rows"], r["cfg"], r["fwd_ms"], r["t_ms"], r["pass_ms"]))
PY
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_kb -o prof -- python3 $GRAFT_REPO_ROOT/scripts/kbench.py --rows 16000000 --layout tiled --reps 5 --tl-configs "2,4,0,1" > $GRAFT_REPO_ROOT/gpurun_out/prof_kb.log 2>&1 || { echo "prof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof_kb.log; exit 1; }
cd $GRAFT_REPO_ROOT && python scripts/prof_summary.py $(find /tmp/prof_kb -name "*.db" | head -1) gpurun_out/kb_kernel_stats.md "kbench 16M rows tiled, 1M-row chunks, multi fwd" > /dev/null && cat gpurun_out/kb_kernel_stats.md
