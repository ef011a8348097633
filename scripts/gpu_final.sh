#!/bin/bash
# End-of-round validation: GPU test tier, smoke, headline bench, kernel-trace profile of a 32M-row bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -40 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.log || { echo "bench failed"; tail -30 gpurun_out/bench_full.log; exit 1; }
cat gpurun_out/bench_full.json
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/proff -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --rows-per-gpu 32000000 --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/proff.log 2>&1 || { echo "prof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/proff.log; exit 1; }
echo profiled
