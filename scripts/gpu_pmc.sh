#!/bin/bash
# PMC counter passes over the kernel microbench (each pass its own rocprofv3 run; no tracing domains with --pmc)
set -o pipefail
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VMEM_RD" \
            "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" \
            "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCC_HIT_sum TCC_MISS_sum" \
            "TCC_EA0_RDREQ_sum TCC_TAG_STALL_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE MeanOccupancyPerActiveCU"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $ctrs -d gpurun_out/pmc2/p$i -o p --output-format csv -- python3 scripts/kbench.py --rows 4000000 --reps 1 > gpurun_out/pmc2/kb$i.json 2> gpurun_out/pmc2/kb$i.log || { echo "pass $i failed"; tail -5 gpurun_out/pmc2/kb$i.log; }
done
ls -R gpurun_out/pmc2 | head -30
