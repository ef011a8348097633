#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python __graft_entry__.py build > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 900 python bench.py > gpurun_out/bench_tiled.json 2> gpurun_out/bench_tiled.log || { echo "bench failed"; tail -40 gpurun_out/bench_tiled.log; exit 1; }
cat gpurun_out/bench_tiled.json
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_tl -o prof -- python3 $GRAFT_REPO_ROOT/scripts/kbench.py --rows 16000000 --layout tiled --configs "0,0,0" > $GRAFT_REPO_ROOT/gpurun_out/prof_tl.log 2>&1 || { echo "prof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof_tl.log; exit 1; }
echo prof ok
