#!/bin/bash
# Row-space class launch order A/B on game5pl (ascending n vs widest first), alternating runs on one box.
set -o pipefail
out=gpurun_out/${1:-rsorder}
mkdir -p $out
export TMPDIR=/tmp
for i in 1 2; do
  for o in asc desc; do
    PML_RS_CLASS_ORDER=$o timeout -k 10 400 python -u bench_game.py --config game5pl --steps 5 --warmup 2 > $out/g_${o}_$i.json 2> $out/g_${o}_$i.log || { echo "bench $o failed"; tail -30 $out/g_${o}_$i.log; exit 1; }
    echo "$o $i: $(grep -o '"coordinate_ms[^}]*}' $out/g_${o}_$i.json) $(grep -o 'sweeps (ms).*' $out/g_${o}_$i.log)"
  done
done
