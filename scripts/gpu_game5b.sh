#!/bin/bash
# Fused segmented CG: kernel + GAME tests, config-5 profile (250k entities) and full config-5 bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python __graft_entry__.py build > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_game_gpu.py -x -q > gpurun_out/pytest_k.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_k.log; exit 1; }
tail -1 gpurun_out/pytest_k.log
cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d /tmp/prof_g5 -o prof -- python3 $GRAFT_REPO_ROOT/bench_game.py --config game5 --entities-per-gpu 250000 --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_g5.log 2>&1 || { echo "prof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof_g5.log; exit 1; }
cd $GRAFT_REPO_ROOT && python scripts/prof_summary.py $(find /tmp/prof_g5 -name "*.db" | head -1) gpurun_out/game5_kernel_stats.md "bench_game.py --config game5 --entities-per-gpu 250000 --steps 2 --warmup 1 (fused CG)" 30 > /dev/null && head -24 gpurun_out/game5_kernel_stats.md
timeout -k 10 1000 python bench_game.py --config game5 --steps 2 --warmup 1 > gpurun_out/bench_game5.json 2> gpurun_out/bench_game5.err || { echo "game5 failed"; tail -20 gpurun_out/bench_game5.err; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_game5.err | tail -4; cat gpurun_out/bench_game5.json
