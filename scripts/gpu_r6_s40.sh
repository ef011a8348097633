#!/bin/bash
# Round 6 step 40: what the row-space / fused-primal overlap buys on game5pl fp64 (PML_RE_OVERLAP=0: the row-space
# classes after the lean launch on one stream).
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6s40
mkdir -p $out
export TMPDIR=/tmp
cd $R
for v in 1 0 1 0; do
  PML_RE_OVERLAP=$v timeout -k 10 240 python3 bench_game.py --config game5pl --precision f64 --steps 3 --warmup 2 > $out/g_$v.json 2> $out/g_$v.log || { echo "game $v failed"; tail -20 $out/g_$v.log; exit 1; }
  python3 - "overlap=$v" "$out/g_$v.json" <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(sys.argv[1], "ms/sweep %.2f median %.2f" % (j["ms_per_step"], j["sweep_ms_median"]), {k: round(v, 2) for k, v in j["coordinate_ms"].items()})
PY
done
