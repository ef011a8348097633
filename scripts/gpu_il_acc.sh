#!/bin/bash
# Interleaved TL: fp64 vs fp32 LDS accumulators x forward block size (16M rows).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "1 10" "0 10" "0 11" "0 12"; do
  set -- $cfg
  PML_TL_ACC64=$1 PML_TL_RBITS=$2 timeout -k 10 300 python scripts/kbench.py --rows 16000000 --chunk-rows 1048576 --il 1 --tl-configs "2,4,0,1,0" > gpurun_out/kb_acc_$1_$2.jsonl 2> gpurun_out/kb_acc_$1_$2.log || { echo "kbench failed $cfg"; tail -30 gpurun_out/kb_acc_$1_$2.log; exit 1; }
  python3 - "$1" "$2" gpurun_out/kb_acc_$1_$2.jsonl <<'PY'
import json, sys
for line in open(sys.argv[3]):
    r = json.loads(line)
    print("acc64=%s rbits=%s fwd %.3f t %.3f pass %.3f" % (sys.argv[1], sys.argv[2], r["fwd_ms"], r["t_ms"], r["pass_ms"]))
PY
done
