#!/bin/bash
# Round 6 step 24: non-temporal row-stream loads in the lean RE kernel (RE_NT=1) vs the production build: the
# 43K-entity micro, then game5pl fp64 RE coordinate. Libraries built in-tree under ops/_lib/exp/.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6s24
mkdir -p $out
export TMPDIR=/tmp
cd $R
for rep in 1 2; do
  for v in base nt; do
    PML_BENCH_QUAD=1 PML_RE_LIB=photon_ml_amd/ops/_lib/exp/libpml_re_$v.so timeout -k 10 240 \
      python3 -u scripts/re_fused_bench.py 43000 lean > $out/micro_$v.$rep.log 2>&1 || { echo "$v micro failed"; tail -20 $out/micro_$v.$rep.log; exit 1; }
    echo "== micro $v rep $rep"; grep -v amdgpu.ids $out/micro_$v.$rep.log | tail -2
  done
done
for rep in 1 2; do
  for v in base nt; do
    PML_RE_LIB=photon_ml_amd/ops/_lib/exp/libpml_re_$v.so timeout -k 10 240 python3 bench_game.py --config game5pl --precision f64 --steps 5 --warmup 2 > $out/g_$v.$rep.json 2> $out/g_$v.$rep.log || { echo "game $v failed"; tail -20 $out/g_$v.$rep.log; exit 1; }
    python3 - "$v" "$out/g_$v.$rep.json" <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print("game", sys.argv[1], "ms/sweep %.2f median %.2f" % (j["ms_per_step"], j["sweep_ms_median"]), {k: round(v, 2) for k, v in j["coordinate_ms"].items()})
PY
  done
done
