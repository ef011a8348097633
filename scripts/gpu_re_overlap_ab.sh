#!/bin/bash
# Row-space / fused-primal overlap A/B on game5pl (PML_RE_OVERLAP 1 vs 0), alternating.
set -o pipefail
out=gpurun_out/${1:-reovl}
mkdir -p $out
export TMPDIR=/tmp
for i in 1 2; do
  for o in 1 0; do
    PML_RE_OVERLAP=$o timeout -k 10 300 python -u bench_game.py --config game5pl --steps 5 --warmup 2 > $out/g_${o}_$i.json 2> $out/g_${o}_$i.log || { echo "bench $o failed"; tail -30 $out/g_${o}_$i.log; exit 1; }
    echo "overlap $o run $i: $(grep -o '"coordinate_ms[^}]*}' $out/g_${o}_$i.json) $(grep -o 'sweeps (ms).*' $out/g_${o}_$i.log)"
  done
done
