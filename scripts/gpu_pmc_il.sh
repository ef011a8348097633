#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel trace only) over the interleaved TL kernels (4M rows).
set -o pipefail
mkdir -p gpurun_out/pmc_il
export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VMEM_RD" \
            "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU" \
            "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCC_HIT_sum TCC_MISS_sum" \
            "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_TAG_STALL_sum" \
            "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctrs -d gpurun_out/pmc_il/p$i -o p --output-format csv -- python3 scripts/kbench.py --rows 4000000 --reps 1 --il 1 --tl-configs "2,4,0,1,0" > gpurun_out/pmc_il/kb$i.json 2> gpurun_out/pmc_il/kb$i.log || echo "pass $i failed: $(grep -i 'error' gpurun_out/pmc_il/kb$i.log | head -2)"
done
python scripts/pmc_summary.py gpurun_out/pmc_il "tl_" gpurun_out/pmc_il_summary.txt > /dev/null
find gpurun_out/pmc_il -name "*.csv" -size +20M -delete
head -80 gpurun_out/pmc_il_summary.txt
