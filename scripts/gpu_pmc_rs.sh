#!/bin/bash
# PMC passes over rs_tron_kernel (1.25M problems of 20 x 20) for the roofline note.
set -o pipefail
out=gpurun_out/pmc_rs
mkdir -p $out
export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 GRBM_GUI_ACTIVE" \
            "FETCH_SIZE SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 150 rocprofv3 --kernel-trace --pmc $ctrs -d $out/p$i -o p --output-format csv -- python3 scripts/rs_tron_bench.py 1250000 20 > $out/rs$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/rs$i.log; }
done
python scripts/pmc_summary.py $out "rs_tron_kernel" $out/summary.txt
find $out -name "*.csv" -size +20M -delete
cat $out/summary.txt
grep -h "rs_tron_kernel" $out/p1/*kernel_trace.csv | cut -c1-400 | tail -3 || true
