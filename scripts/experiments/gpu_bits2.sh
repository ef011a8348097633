#!/bin/bash
# Forward block size sweep with fp32 LDS accumulators (kernel microbench, 16M rows), one process per layout.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/kbench_bits2.jsonl
for rc in "10 1" "10 0" "11 0" "12 0"; do
  set -- $rc
  PML_TL_RBITS=$1 PML_TL_ACC64=$2 timeout -k 10 300 python scripts/kbench.py --rows 16000000 --reps 5 --configs "0,1,0" > gpurun_out/kb_b2_$1_$2.json 2> gpurun_out/kb_b2_$1_$2.log || { echo "kbench $1 $2 failed"; tail -20 gpurun_out/kb_b2_$1_$2.log; exit 1; }
  python -c "import json,sys; r=json.load(open('gpurun_out/kb_b2_$1_$2.json')); print('rbits $1 acc64 $2 fwd %.3f t %.3f narrow %.3f' % (r['fwd_ms'], r['t_ms'], r['narrow_frac_fwd']))"
done
