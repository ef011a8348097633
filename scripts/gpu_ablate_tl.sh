#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python __graft_entry__.py build > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 400 python scripts/kbench.py --rows 16000000 --layout tiled --configs "0,0,0" --ablate 0 1 2 4 3 6 > gpurun_out/abl_tl.log 2>&1 || { echo "kbench failed"; tail -30 gpurun_out/abl_tl.log; exit 1; }
python3 - <<'PY'
import json
for line in open("gpurun_out/abl_tl.log"):
    if line.startswith("{"):
        r = json.loads(line); print("ablate %d: fwd %.3f t %.3f" % (r["ablate"], r["fwd_ms"], r["t_ms"]))
PY
