#!/bin/bash
# Headline bench under the TL kernel knobs (waves per work-group, transpose item size).
set -o pipefail
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 900 python bench.py > gpurun_out/knob_$tag.json 2> gpurun_out/knob_$tag.log || { echo "bench $tag failed"; tail -20 gpurun_out/knob_$tag.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/knob_$tag.json'));print('$tag', round(d['ms_per_step'],2))"
}
run base PML_TL_WAVES=2
run fwd_w4 PML_TL_WAVES=4
run t_w2 PML_TL_WAVES_T=2
run items64k PML_TL_ITEM_ENTRIES=65536
run items256k PML_TL_ITEM_ENTRIES=262144
PML_SYNC_TIMING=1 timeout -k 10 900 python -u bench_game.py --config game5 --steps 3 --warmup 2 --log-level DEBUG > gpurun_out/g5dbg.json 2> gpurun_out/g5dbg.log || { echo "game5 failed"; tail -20 gpurun_out/g5dbg.log; exit 1; }
grep -E "Update coordinate|Coordinate descent iteration|row-space" gpurun_out/g5dbg.log | tail -12 | cut -c1-200
cat gpurun_out/g5dbg.json | cut -c1-200
