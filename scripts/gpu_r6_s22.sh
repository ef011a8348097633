#!/bin/bash
# Round 6 step 22: row-space class launch order A/B on game5pl (fp64 FE): the RE coordinate's tail after the lean launch.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6s22
mkdir -p $out
export TMPDIR=/tmp
cd $R
for rep in 1 2; do
for v in desc small_first:12 small_first:16 asc; do
  ord=${v%%:*}; sn=${v##*:}; [ "$sn" = "$v" ] && sn=12
  PML_RS_CLASS_ORDER=$ord PML_RS_SMALL_N=$sn timeout -k 10 240 python3 bench_game.py --config game5pl --precision f64 --steps 5 --warmup 2 > $out/$ord$sn.$rep.json 2> $out/$ord$sn.$rep.log || { echo "run $v failed"; tail -20 $out/$ord$sn.$rep.log; exit 1; }
  python3 - "$v" "$out/$ord$sn.$rep.json" <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(sys.argv[1], "ms/sweep %.2f median %.2f" % (j["ms_per_step"], j["sweep_ms_median"]), {k: round(v, 2) for k, v in j["coordinate_ms"].items()})
PY
done
done
