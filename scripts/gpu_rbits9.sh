#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rb in 10 9; do
  PML_TL_RBITS=$rb timeout -k 10 300 python scripts/kbench.py --rows 16000000 --chunk-rows 1048576 --il 1 --tl-configs "2,4,0,1,0;4,4,0,1,0;1,4,0,1,0" > gpurun_out/kb_rb_$rb.jsonl 2> gpurun_out/kb_rb_$rb.log || { echo "kbench failed $rb"; tail -30 gpurun_out/kb_rb_$rb.log; exit 1; }
  python3 - "$rb" gpurun_out/kb_rb_$rb.jsonl <<'PY'
import json, sys
for line in open(sys.argv[2]):
    r = json.loads(line)
    print("rbits=%s cfg=%s fwd %.3f t %.3f pass %.3f" % (sys.argv[1], r["cfg"][1:3], r["fwd_ms"], r["t_ms"], r["pass_ms"]))
PY
done
