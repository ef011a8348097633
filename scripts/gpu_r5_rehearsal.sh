#!/bin/bash
# Round 5: 2-rank data-parallel + entity-sharded GAME rehearsal on ONE GPU (both ranks on cuda:0, gloo collectives)
# at the game5pl shape with 500K entities per rank (two full game5pl ranks do not fit one GPU), with entity-aligned row placement at ingest (default) and without (per-update
# routing). -> gpurun_out/r5rehearsal/
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5rehearsal
mkdir -p $out
for mode in placed routed; do
  extra=""; [ $mode = routed ] && extra="--no-placement"
  PML_DIST_BACKEND=gloo timeout -k 10 1100 python -u bench_game.py --gpus 2 --rehearsal --config game5pl --entities-per-gpu ${ENT:-500000} --steps 2 --warmup 1 --log-level INFO $extra > $out/$mode.json 2> $out/$mode.log || { echo "$mode failed"; tail -40 $out/$mode.log; exit 1; }
  echo "== $mode"; grep -E "rows placed|route rows|coordinates built|sweeps \(ms\)" $out/$mode.log | cut -c1-300
  grep -o '"coordinate_ms[^}]*}\|"routed_bytes_per_update[^}]*}\|"placement_s[^,]*\|"ms_per_step[^,]*' $out/$mode.json
done
