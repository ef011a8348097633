#!/bin/bash
# GAME after size classes + seg_gram: GPU tests, then both config-5 presets with phase timings.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_game_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_game4.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_game4.log; exit 1; }
tail -2 gpurun_out/pytest_game4.log
for cfg in game5pl game5; do
  PML_SYNC_TIMING=1 PML_TRON_STATS=1 timeout -k 10 900 python -u bench_game.py --config $cfg --steps 3 --warmup 2 --log-level DEBUG > gpurun_out/bench_${cfg}_v4.json 2> gpurun_out/bench_${cfg}_v4.log || { echo "bench $cfg failed"; tail -30 gpurun_out/bench_${cfg}_v4.log; exit 1; }
  grep -E "generated|built|row-space|primal|coordinate (global|per-entity)|RE stats|allocator|Timed|setup" gpurun_out/bench_${cfg}_v4.log | cut -c1-250 | tail -40
  cat gpurun_out/bench_${cfg}_v4.json
done
