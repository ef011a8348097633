#!/bin/bash
# Block / tile size sweep of the tiled layout (kernel microbench, 16M rows), one process per layout.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/kbench_bits.jsonl
for rc in "10 10" "11 10" "10 11" "11 11"; do
  set -- $rc
  PML_TL_RBITS=$1 PML_TL_CBITS=$2 timeout -k 10 300 python scripts/kbench.py --rows 16000000 --reps 5 --configs "0,1,0" > gpurun_out/kb_bits_$1_$2.json 2> gpurun_out/kb_bits_$1_$2.log || { echo "kbench $1 $2 failed"; tail -20 gpurun_out/kb_bits_$1_$2.log; exit 1; }
  echo "{\"rbits\": $1, \"cbits\": $2, \"r\": $(cat gpurun_out/kb_bits_$1_$2.json)}" >> gpurun_out/kbench_bits.jsonl
done
cat gpurun_out/kbench_bits.jsonl
