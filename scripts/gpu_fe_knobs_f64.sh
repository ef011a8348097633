#!/bin/bash
# Tiled-layout knobs for the fp64 GAME fixed-effect shard (game5pl at fp64 FE features): FE coordinate ms.
set -o pipefail
out=gpurun_out/${1:-feknobs64}
mkdir -p $out
export TMPDIR=/tmp
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench_game.py --config game5pl --precision f64 --steps 3 --warmup 2 > $out/g_$tag.json 2> $out/g_$tag.log || { echo "$tag failed"; tail -20 $out/g_$tag.log; return 1; }
  echo "$tag: $(grep -o '"coordinate_ms[^}]*}' $out/g_$tag.json)"
}
run auto PML_X=1 && run cb11_it64k PML_TL_CBITS=11 PML_TL_ITEM_ENTRIES=65536 && \
run cb11_it256k PML_TL_CBITS=11 PML_TL_ITEM_ENTRIES=262144 && run cb10_it128k PML_TL_CBITS=10 PML_TL_ITEM_ENTRIES=131072 && \
run auto_rb9 PML_TL_RBITS=9 && run auto_rb11 PML_TL_RBITS=11 && run auto2 PML_X=1
