#!/bin/bash
# A/B on one box: L-BFGS two-loop + history pair as HIP kernels (default) vs torch launches; and whether the
# rocprofv3 exit-time crash follows the cooperative launch.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
for v in 1 0 1 0; do
  PML_LBFGS_NATIVE_TWO_LOOP=$v timeout -k 10 600 python -u bench_game.py --config game5 --steps 3 --warmup 2 > gpurun_out/ab_g5_$v.json 2> gpurun_out/ab_g5_$v.log || { echo "game5 $v failed"; tail -20 gpurun_out/ab_g5_$v.log; exit 1; }
  echo "native_two_loop=$v $(grep -E 'iteration 2 coordinate global' gpurun_out/ab_g5_$v.log | tail -1) $(cut -c150-200 gpurun_out/ab_g5_$v.json)"
done
cd /tmp
PML_LBFGS_NATIVE_TWO_LOOP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_t0 -o prof -- python3 $R/bench.py --steps 2 --warmup 1 --rows-per-gpu 4000000 > $R/gpurun_out/prof_t0.json 2> $R/gpurun_out/prof_t0.log; echo "rocprof native=0 rc=$?"
PML_LBFGS_NATIVE_TWO_LOOP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_t1 -o prof -- python3 $R/bench.py --steps 2 --warmup 1 --rows-per-gpu 4000000 > $R/gpurun_out/prof_t1.json 2> $R/gpurun_out/prof_t1.log; echo "rocprof native=1 rc=$?"
rm -rf $R/gpurun_out/prof_t0 $R/gpurun_out/prof_t1
