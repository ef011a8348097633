#!/bin/bash
# Row-chunk size sweep of the headline bench (fewer per-(chunk, tile) transpose items and partial rows).
set -o pipefail
mkdir -p gpurun_out
for c in 524288 262144; do
  timeout -k 10 900 python bench.py --chunk-rows $c > gpurun_out/bench_chunk_$c.json 2> gpurun_out/bench_chunk_$c.log || { echo "bench $c failed"; tail -30 gpurun_out/bench_chunk_$c.log; exit 1; }
  echo "chunk_rows=$c"; cat gpurun_out/bench_chunk_$c.json | cut -c1-230
done
