#!/bin/bash
# Headline bench (N=1) + kernel-trace profile of a 32M-row run.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.log || { echo "full bench failed"; tail -40 gpurun_out/bench_full.log; exit 1; }
cat gpurun_out/bench_full.json
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/profb -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --rows-per-gpu 32000000 --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/profb.log 2>&1 || { echo "prof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/profb.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/profb -name "*kernel_stats.csv" | head -3
