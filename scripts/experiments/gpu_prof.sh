#!/bin/bash
# Narrow-round A/B (kernel microbench, 16M rows) + kernel-trace profile of the bench at 32M rows.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python scripts/kbench.py --rows 16000000 --reps 5 --configs "0,1,0" --narrow 0 1 > gpurun_out/kbench_narrow_16M.jsonl 2> gpurun_out/kbench_narrow.log || { echo "kbench failed"; tail -30 gpurun_out/kbench_narrow.log; exit 1; }
cat gpurun_out/kbench_narrow_16M.jsonl
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_narrow -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --rows-per-gpu 32000000 --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_narrow.log 2>&1 || { echo "prof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof_narrow.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof_narrow -name "*kernel_stats.csv" | head -3
