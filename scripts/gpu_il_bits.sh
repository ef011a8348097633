#!/bin/bash
# Interleaved TL layout: block/tile size sweep (rbits x cbits) on 16M rows, 2-wave forward / 4-wave transpose.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "10 10" "11 10" "10 11" "11 11" "10 9"; do
  set -- $cfg
  PML_TL_RBITS=$1 PML_TL_CBITS=$2 timeout -k 10 300 python scripts/kbench.py --rows 16000000 --chunk-rows 1048576 --il 1 --tl-configs "2,4,0,1,0;2,2,0,1,0" > gpurun_out/kb_il_$1_$2.jsonl 2> gpurun_out/kb_il_$1_$2.log || { echo "kbench failed $cfg"; tail -30 gpurun_out/kb_il_$1_$2.log; exit 1; }
  python3 - "$1" "$2" gpurun_out/kb_il_$1_$2.jsonl <<'PY'
import json, sys
for line in open(sys.argv[3]):
    r = json.loads(line)
    print("rbits=%s cbits=%s cfg=%s fwd %.3f t %.3f pass %.3f" % (sys.argv[1], sys.argv[2], r["cfg"][1:3], r["fwd_ms"], r["t_ms"], r["pass_ms"]))
PY
done
