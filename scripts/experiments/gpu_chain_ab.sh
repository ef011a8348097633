#!/bin/bash
# A/B on one box: L-BFGS two-loop as the C++-launched step-kernel chain (default) vs the torch recursion.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 1 0 1 0; do
  PML_LBFGS_NATIVE_TWO_LOOP=$v timeout -k 10 600 python -u bench_game.py --config game5 --steps 3 --warmup 2 > gpurun_out/abc_g5_$v.json 2> gpurun_out/abc_g5_$v.log || { echo "game5 $v failed"; tail -20 gpurun_out/abc_g5_$v.log; exit 1; }
  echo "native_two_loop=$v $(grep -E 'iteration 2 coordinate global' gpurun_out/abc_g5_$v.log | tail -1) $(cut -c150-200 gpurun_out/abc_g5_$v.json)"
done
for v in 1 0; do
  PML_LBFGS_NATIVE_TWO_LOOP=$v timeout -k 10 600 python bench.py > gpurun_out/abc_bench_$v.json 2> gpurun_out/abc_bench_$v.log || { echo "bench $v failed"; exit 1; }
  echo "native_two_loop=$v bench $(cut -c150-220 gpurun_out/abc_bench_$v.json)"
done
