#!/bin/bash
# Interleaved TL stream ablation: 0 = full, 8 = no gathers, 16 = no LDS adds, 24 = neither (16M rows).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python scripts/kbench.py --rows 16000000 --chunk-rows 1048576 --il 1 --ablate 0 8 16 24 --tl-configs "2,4,0,1,0" > gpurun_out/kbench_abl.jsonl 2> gpurun_out/kbench_abl.log || { tail -30 gpurun_out/kbench_abl.log; exit 1; }
python3 - <<'PY'
import json
for line in open("gpurun_out/kbench_abl.jsonl"):
    r = json.loads(line)
    print("ablate=%d fwd %.3f (%.0f GB/s) t %.3f (%.0f GB/s)" % (r["ablate"], r["fwd_ms"], r["fwd_GBps"], r["t_ms"], r["t_GBps"]))
PY
