#!/bin/bash
# PMC passes over the tiled kernels (each pass its own rocprofv3 run; kernel-trace only alongside --pmc).
set -o pipefail
mkdir -p gpurun_out/pmc_tl
export TMPDIR=/tmp
python __graft_entry__.py build > gpurun_out/build.log 2>&1 || { echo "build failed"; exit 1; }
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VMEM_RD" \
            "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU" \
            "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCC_HIT_sum TCC_MISS_sum" \
            "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_TAG_STALL_sum MeanOccupancyPerActiveCU"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $ctrs -d gpurun_out/pmc_tl/p$i -o p --output-format csv -- python3 scripts/kbench.py --rows 4000000 --reps 1 > gpurun_out/pmc_tl/kb$i.json 2> gpurun_out/pmc_tl/kb$i.log || { echo "pass $i failed"; tail -5 gpurun_out/pmc_tl/kb$i.log; }
done
python scripts/pmc_summary.py gpurun_out/pmc_tl "tl_" gpurun_out/pmc_tl_summary.txt
find gpurun_out/pmc_tl -name "*.csv" -size +20M -delete
