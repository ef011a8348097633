#!/bin/bash
# Transpose item size sweep at 125M rows.
set -o pipefail
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 900 python bench.py > gpurun_out/knob_$tag.json 2> gpurun_out/knob_$tag.log || { echo "bench $tag failed"; tail -20 gpurun_out/knob_$tag.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/knob_$tag.json'));print('$tag', round(d['ms_per_step'],2))"
}
run items256k_b PML_TL_ITEM_ENTRIES=262144
run items512k PML_TL_ITEM_ENTRIES=524288
run items1m PML_TL_ITEM_ENTRIES=1048576
run base_b PML_TL_WAVES=2
