#!/bin/bash
# Entity-masked block-diagonal passes: bitwise test, then game5pl with CG activity stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_game_gpu.py -x -q --timeout 300 --timeout-method thread -k "masked or segmented or row_space" > gpurun_out/pytest_game5.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_game5.log; exit 1; }
tail -2 gpurun_out/pytest_game5.log
PML_SYNC_TIMING=1 PML_TRON_STATS=1 timeout -k 10 900 python -u bench_game.py --config game5pl --steps 3 --warmup 2 --log-level DEBUG > gpurun_out/bench_game5pl_v6.json 2> gpurun_out/bench_game5pl_v6.log || { echo "bench failed"; tail -30 gpurun_out/bench_game5pl_v6.log; exit 1; }
grep -E "entity-masked|primal|block-diagonal TRON|coordinate (global|per-entity)|allocator" gpurun_out/bench_game5pl_v6.log | cut -c1-250 | tail -14
cat gpurun_out/bench_game5pl_v6.json
