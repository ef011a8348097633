#!/bin/bash
# Tiled-layout knobs for the GAME fixed-effect shard (game5pl: 25M rows x 30 nnz, 1M features): FE coordinate ms.
set -o pipefail
out=gpurun_out/${1:-feknobs}
mkdir -p $out
export TMPDIR=/tmp
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench_game.py --config game5pl --steps 3 --warmup 2 > $out/g_$tag.json 2> $out/g_$tag.log || { echo "$tag failed"; tail -20 $out/g_$tag.log; return 1; }
  echo "$tag: $(grep -o '"coordinate_ms[^}]*}' $out/g_$tag.json)"
}
run base PML_TL_ITEM_ENTRIES=262144 && run it64k PML_TL_ITEM_ENTRIES=65536 && run it128k PML_TL_ITEM_ENTRIES=131072 && \
run it512k PML_TL_ITEM_ENTRIES=524288 && run cb9 PML_TL_CBITS=9 && run cb11 PML_TL_CBITS=11 && run rb9 PML_TL_RBITS=9 && \
run rb11 PML_TL_RBITS=11 && run base2 PML_TL_ITEM_ENTRIES=262144
