#!/bin/bash
# Headline timed window (125M rows x 1M features, 5 timed L-BFGS steps): rocprofv3 kernel + marker trace,
# kernel-busy share, top kernels and idle gaps of the "bench timed steps" region.
set -o pipefail
R=$GRAFT_REPO_ROOT
tag=${1:-r3}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
PML_TRACE=1 timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace -d $R/gpurun_out/prof_hl -o prof -- python3 $R/bench.py --steps 5 --warmup 2 --game off > $R/gpurun_out/prof_hl.json 2> $R/gpurun_out/prof_hl.log || { echo "bench prof failed"; tail -30 $R/gpurun_out/prof_hl.log; exit 1; }
db=$(find $R/gpurun_out/prof_hl -name "*.db" | head -1)
python3 $R/scripts/prof_window.py "$db" "bench timed steps" $R/gpurun_out/bench_125M_timed_window_$tag.md > /dev/null && head -45 $R/gpurun_out/bench_125M_timed_window_$tag.md
rm -rf $R/gpurun_out/prof_hl
