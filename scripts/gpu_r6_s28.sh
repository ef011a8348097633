#!/bin/bash
# Round 6 step 28: lean RE launch order A/B (PML_RE_ORDER: largest first vs the K largest first and then smallest first)
# on game5pl fp64 (RE coordinate ms).
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6s28
mkdir -p $out
export TMPDIR=/tmp
cd $R
for rep in 1 2; do
  for v in desc head:64 head:256 head:768; do
    tag=${v/:/_}
    PML_RE_ORDER=$v timeout -k 10 240 python3 bench_game.py --config game5pl --precision f64 --steps 5 --warmup 2 > $out/g_$tag.$rep.json 2> $out/g_$tag.$rep.log || { echo "game $v failed"; tail -20 $out/g_$tag.$rep.log; exit 1; }
    python3 - "$v" "$out/g_$tag.$rep.json" <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print("game", sys.argv[1], "ms/sweep %.2f median %.2f" % (j["ms_per_step"], j["sweep_ms_median"]), {k: round(v, 2) for k, v in j["coordinate_ms"].items()})
PY
  done
done
