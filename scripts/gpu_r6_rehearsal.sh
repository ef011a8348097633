#!/bin/bash
# Round 6: 2-rank entity-sharded GAME rehearsal on ONE GPU (gloo, both ranks on cuda:0, 500K entities per rank) with
# the final tree, placed at ingest (default); then a 2-rank headline (DP) rehearsal of bench.py at reduced rows.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6rehearsal
mkdir -p $out
PML_DIST_BACKEND=gloo timeout -k 10 600 python -u bench_game.py --gpus 2 --rehearsal --config game5pl --entities-per-gpu 500000 --steps 2 --warmup 1 --log-level INFO > $out/placed.json 2> $out/placed.log || { echo "game rehearsal failed"; tail -40 $out/placed.log; exit 1; }
grep -E "rows placed|coordinates built|sweeps \(ms\)" $out/placed.log | cut -c1-300
grep -o '"coordinate_ms[^}]*}\|"routed_bytes_per_update[^}]*}\|"placement_s[^,]*\|"ms_per_step[^,]*' $out/placed.json
PML_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --rehearsal --rows-per-gpu 8000000 --steps 3 --warmup 2 --game off > $out/headline.json 2> $out/headline.log || { echo "headline rehearsal failed"; tail -30 $out/headline.log; exit 1; }
cat $out/headline.json
