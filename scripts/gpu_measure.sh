#!/bin/bash
# Round measurements: headline bench and GAME config 5 (uniform and power-law entity sizes), no profiler.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-latest}
timeout -k 10 600 python bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.log || { echo "bench failed"; tail -30 gpurun_out/bench_$tag.log; exit 1; }
cut -c1-200 gpurun_out/bench_$tag.json
for cfg in game5 game5pl; do
  timeout -k 10 900 python -u bench_game.py --config $cfg --steps 3 --warmup 2 > gpurun_out/${cfg}_$tag.json 2> gpurun_out/${cfg}_$tag.log || { echo "bench $cfg failed"; tail -30 gpurun_out/${cfg}_$tag.log; exit 1; }
  grep -E "coordinate (global|per-entity)" gpurun_out/${cfg}_$tag.log | tail -2
  cut -c1-200 gpurun_out/${cfg}_$tag.json
done
