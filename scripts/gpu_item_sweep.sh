#!/bin/bash
# Transpose item size sweep on the interleaved TL layout (16M rows).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for it in 32768 65536 131072 262144; do
  PML_TL_ITEM_ENTRIES=$it timeout -k 10 300 python scripts/kbench.py --rows 16000000 --chunk-rows 1048576 --il 1 --tl-configs "2,4,0,1,0;2,2,0,1,0" > gpurun_out/kb_item_$it.jsonl 2> gpurun_out/kb_item_$it.log || { echo "kbench failed $it"; tail -30 gpurun_out/kb_item_$it.log; exit 1; }
  python3 - "$it" gpurun_out/kb_item_$it.jsonl <<'PY'
import json, sys
for line in open(sys.argv[2]):
    r = json.loads(line)
    print("item=%s cfg=%s fwd %.3f t %.3f pass %.3f nblk_t %d" % (sys.argv[1], r["cfg"][1:3], r["fwd_ms"], r["t_ms"], r["pass_ms"], r["nblk_t"]))
PY
done
