#!/bin/bash
# A/B on one box: margin cache shifted across offset changes (default) vs dropped (forward pass per FE update).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 1 0 1 0; do
  PML_OFFSET_SHIFT_CACHE=$v timeout -k 10 600 python -u bench_game.py --config game5 --steps 3 --warmup 2 > gpurun_out/abz_g5_$v.json 2> gpurun_out/abz_g5_$v.log || { echo "game5 $v failed"; tail -20 gpurun_out/abz_g5_$v.log; exit 1; }
  echo "offset_shift_cache=$v $(grep -E 'fixed effect per sweep' gpurun_out/abz_g5_$v.log | tail -1) $(grep -E 'iteration 2 coordinate global' gpurun_out/abz_g5_$v.log | tail -1) $(cut -c150-200 gpurun_out/abz_g5_$v.json)"
done
