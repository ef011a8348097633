#!/bin/bash
# Round 6 step 36: fixed-effect TL kernel knobs at fp64 feature storage (experiment build libpml_glm_abl.so, runtime
# knobs): waves per forward / transpose workgroup and the stream-pipeline depth, game5pl fp64 FE coordinate ms.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6s36
mkdir -p $out
export TMPDIR=/tmp
cd $R
export PML_GLM_LIB=photon_ml_amd/ops/_lib/libpml_glm_abl.so
for v in "base" "PML_TL_DEEP=1" "PML_TL_DEEP=2" "PML_TL_DEEP_T=1" "PML_TL_DEEP_T=2" "PML_TL_WAVES=4" "PML_TL_WAVES_T=2" "base"; do
  tag=${v//=/_}
  env $( [ "$v" = base ] || echo "$v" ) timeout -k 10 240 python3 bench_game.py --config game5pl --precision f64 --steps 3 --warmup 2 > $out/g_$tag.json 2> $out/g_$tag.log || { echo "game $v failed"; tail -20 $out/g_$tag.log; exit 1; }
  python3 - "$v" "$out/g_$tag.json" <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(sys.argv[1], "ms/sweep %.2f median %.2f" % (j["ms_per_step"], j["sweep_ms_median"]), {k: round(v, 2) for k, v in j["coordinate_ms"].items()})
PY
done
