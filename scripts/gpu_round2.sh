#!/bin/bash
# GPU validation round 2: all gpu tests (kernels + GAME), smoke, full bench, kernel-trace profile of the bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python __graft_entry__.py build > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 900 python -m pytest tests/ -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -40 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 900 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.log || { echo "full bench failed"; tail -40 gpurun_out/bench_full.log; exit 1; }
cat gpurun_out/bench_full.json
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof2 -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --rows-per-gpu 32000000 --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof2.log 2>&1 || { echo "prof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof2.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof2 -name "*kernel_stats.csv" | head -3
