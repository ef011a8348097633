#!/bin/bash
# Round 5: which entities the row space should take now that the lean primal kernel is faster — game5pl with the
# row-space upper bound PML_RS_NMAX and the dense-class ratio PML_RS_BIG_NNZ_RATIO varied (5 timed sweeps each).
set -o pipefail
out=gpurun_out/r5rsmix
mkdir -p $out
export TMPDIR=/tmp
run() {  # tag env...
  tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench_game.py --config game5pl --steps 5 --warmup 2 > $out/$tag.json 2> $out/$tag.log || { echo "$tag failed"; tail -30 $out/$tag.log; exit 1; }
  echo "$tag: $(grep -o '"coordinate_ms[^}]*}' $out/$tag.json) $(grep -o 'sweeps (ms).*' $out/$tag.log)"
}
run base PML_RS_NMAX=128 && run nobig PML_RS_BIG_NNZ_RATIO=100 && run n48 PML_RS_NMAX=48 && run n32 PML_RS_NMAX=32 && run base2 PML_RS_NMAX=128
