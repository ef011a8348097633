#!/bin/bash
# Round 6 step 41: row-space / primal split by rows per entity (PML_RS_NMAX) on game5pl fp64, RE ms.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6s41
mkdir -p $out
export TMPDIR=/tmp
cd $R
for v in 128 64 96 160 128; do
  PML_RS_NMAX=$v timeout -k 10 240 python3 bench_game.py --config game5pl --precision f64 --steps 3 --warmup 2 > $out/g_$v.json 2> $out/g_$v.log || { echo "game $v failed"; tail -20 $out/g_$v.log; exit 1; }
  python3 - "nmax=$v" "$out/g_$v.json" <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(sys.argv[1], "ms/sweep %.2f median %.2f" % (j["ms_per_step"], j["sweep_ms_median"]), {k: round(v, 2) for k, v in j["coordinate_ms"].items()}, j.get("re_solver_routing", {}).get("row_space"))
PY
done
