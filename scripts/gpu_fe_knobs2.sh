#!/bin/bash
# Column-tile bits x item size for the GAME FE shard, and cbits 11 on the headline shape.
set -o pipefail
out=gpurun_out/${1:-feknobs2}
mkdir -p $out
export TMPDIR=/tmp
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench_game.py --config game5pl --steps 3 --warmup 2 > $out/g_$tag.json 2> $out/g_$tag.log || { echo "$tag failed"; tail -20 $out/g_$tag.log; return 1; }
  echo "$tag: $(grep -o '"coordinate_ms[^}]*}' $out/g_$tag.json)"
}
hl() {
  local tag=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --game off > $out/h_$tag.json 2> $out/h_$tag.log || { echo "hl $tag failed"; tail -20 $out/h_$tag.log; return 1; }
  echo "headline $tag: $(grep -o '"ms_per_step": [0-9.]*' $out/h_$tag.json)"
}
run cb11_it128k PML_TL_CBITS=11 PML_TL_ITEM_ENTRIES=131072 && run cb11_it64k PML_TL_CBITS=11 PML_TL_ITEM_ENTRIES=65536 && \
run cb11_it512k PML_TL_CBITS=11 PML_TL_ITEM_ENTRIES=524288 && run cb11 PML_TL_CBITS=11 && \
hl cb10 PML_TL_CBITS=10 && hl cb11 PML_TL_CBITS=11 && hl cb11_it512k PML_TL_CBITS=11 PML_TL_ITEM_ENTRIES=524288
