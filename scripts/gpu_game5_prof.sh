#!/bin/bash
# Kernel profile of the config-5-shaped GAME sweep (250k entities x 1001 coefficients, 1 GPU).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python __graft_entry__.py build > gpurun_out/build.log 2>&1 || { echo "build failed"; exit 1; }
cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d /tmp/prof_g5 -o prof -- python3 $GRAFT_REPO_ROOT/bench_game.py --config game5 --entities-per-gpu 250000 --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_g5.log 2>&1 || { echo "prof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof_g5.log; exit 1; }
cd $GRAFT_REPO_ROOT && python scripts/prof_summary.py $(find /tmp/prof_g5 -name "*.db" | head -1) gpurun_out/game5_kernel_stats.md "bench_game.py --config game5 --entities-per-gpu 250000 --steps 2 --warmup 1" 40 > /dev/null && cat gpurun_out/game5_kernel_stats.md
grep -v amdgpu.ids gpurun_out/prof_g5.log | grep bench_game | tail -5
