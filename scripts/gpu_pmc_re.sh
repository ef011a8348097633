#!/bin/bash
# PMC passes over the fused primal TRON microbench (re_tron_csr_kernel).
set -o pipefail
tag=${1:-re}
out=gpurun_out/pmc_$tag
mkdir -p $out
export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE TA_TA_BUSY_sum TD_TD_BUSY_sum" \
            "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
            "FETCH_SIZE TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE" \
            "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $ctrs -d $out/p$i -o p --output-format csv -- python3 scripts/re_fused_bench.py 43000 2 > $out/b$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/b$i.log; exit 1; }
done
python3 scripts/pmc_summary.py $out "re_tron" $out/summary.txt
find $out -name "*.csv" -size +20M -delete
cat $out/summary.txt
