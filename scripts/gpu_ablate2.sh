#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python scripts/kbench.py --rows 8000000 --chunk-rows 1048576 --ablate 0 1 4 8 2 3 --configs "0,0,0;0,0,8192;0,1,0" > gpurun_out/ablate2.jsonl 2> gpurun_out/ablate2.log || { tail -30 gpurun_out/ablate2.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/ablate2.jsonl'):
    r=json.loads(l); print(r['cfg'], r['ablate'], round(r['fwd_ms'],3), round(r['t_ms'],3))
"
