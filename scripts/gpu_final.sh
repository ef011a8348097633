#!/bin/bash
# Round measurements: both GAME config-5 presets and the headline bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in game5 game5pl; do
  timeout -k 10 900 python -u bench_game.py --config $cfg --steps 3 --warmup 2 > gpurun_out/final_$cfg.json 2> gpurun_out/final_$cfg.log || { echo "bench $cfg failed"; tail -30 gpurun_out/final_$cfg.log; exit 1; }
  grep -E "built in|coordinate (global|per-entity)" gpurun_out/final_$cfg.log | tail -3
  cat gpurun_out/final_$cfg.json | cut -c1-240
done
timeout -k 10 900 python bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.log || { echo "bench failed"; tail -30 gpurun_out/final_bench.log; exit 1; }
cat gpurun_out/final_bench.json | cut -c1-240
