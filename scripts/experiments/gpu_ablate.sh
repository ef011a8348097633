#!/bin/bash
# Ablations of the TL streams (experiment build, scripts/kbench.py --ablate): 0 none, 1 no LDS atomics,
# 2 no gathers / key-window loads, 4 fp32 products, 3 = 1|2.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
PML_GLM_LIB=$PWD/photon_ml_amd/ops/_lib/libpml_glm_abl.so timeout -k 10 400 python scripts/kbench.py --rows 16000000 --reps 5 --configs "0,1,0" --ablate 0 2 8 16 24 > gpurun_out/kbench_ablate.jsonl 2> gpurun_out/kbench_ablate.log || { echo "kbench failed"; tail -30 gpurun_out/kbench_ablate.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/kbench_ablate.jsonl"):
    r = json.loads(l)
    print(r["ablate"], "fwd %.3f ms  t %.3f ms" % (r["fwd_ms"], r["t_ms"]))
PY
