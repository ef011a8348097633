#!/bin/bash
# Round 5 (after the quad-pass fixes): PMC passes of the lean streaming RE kernel on 43K game5pl-like entities (what bounds it: LDS, TA,
# HBM, or waits), plus a plain timing run. -> gpurun_out/r5leanpmc/summary.txt
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5leanpmc2
mkdir -p $out
timeout -k 10 240 python3 scripts/re_fused_bench.py 43000 lean > $out/time.log 2>&1 || { echo "timing failed"; tail -5 $out/time.log; exit 1; }
cat $out/time.log
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE TA_TA_BUSY_sum TD_TD_BUSY_sum" \
            "FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE TCP_TCC_READ_REQ_sum" \
            "SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SCRATCH SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctrs -d $out/p$i -o p --output-format csv -- python3 scripts/re_fused_bench.py 43000 lean > $out/b$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $out/b$i.log; exit 1; }
done
python3 scripts/pmc_summary.py $out "re_tron" $out/summary.txt
find $out -name "*.csv" -delete
cat $out/summary.txt
