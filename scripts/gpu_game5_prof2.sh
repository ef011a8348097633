#!/bin/bash
# Kernel-trace profile of the GAME config-5 shape at 250K entities (row-space random-effect solve).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_g5b -o prof -- python3 $GRAFT_REPO_ROOT/bench_game.py --config game5 --entities-per-gpu 250000 --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_g5b.log 2>&1 || { echo "prof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof_g5b.log; exit 1; }
cd $GRAFT_REPO_ROOT && python scripts/prof_summary.py $(find /tmp/prof_g5b -name "*.db" | head -1) gpurun_out/game5_rs_kernel_stats.md "bench_game.py --config game5 --entities-per-gpu 250000 --steps 2 --warmup 1 (row-space RE solve, HIP batched GEMV)" 30 > /dev/null && cat gpurun_out/game5_rs_kernel_stats.md
grep -v amdgpu.ids gpurun_out/prof_g5b.log | grep bench_game | tail -4
