#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "dedup or bucketed" -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_dd.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_dd.log; exit 1; }
tail -1 gpurun_out/pytest_dd.log
timeout -k 10 400 python scripts/kbench.py --rows 16000000 --chunk-rows 1048576 --il 1 --tl-configs "2,4,0,1,0,0,0;2,4,0,1,0,1,0;2,4,0,1,0,0,1;2,4,0,1,0,1,1;2,4,0,1,0,0,0" > gpurun_out/kb_dd.jsonl 2> gpurun_out/kb_dd.log || { tail -30 gpurun_out/kb_dd.log; exit 1; }
python3 - <<'PY'
import json
for line in open("gpurun_out/kb_dd.jsonl"):
    r = json.loads(line)
    print("cfg=%s fwd %.3f t %.3f pass %.3f" % (r["cfg"][1:], r["fwd_ms"], r["t_ms"], r["pass_ms"]))
PY
