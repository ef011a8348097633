#!/bin/bash
# PMC passes over the production-shape headline bench (125M rows/GPU x 1M features x 100 nnz, tiled layout):
# the counters of the tl_fwd_multi / tl_t_multi kernels that the timed L-BFGS steps actually launch.
# Each pass is its own rocprofv3 run (kernel-trace only alongside --pmc, per the pool rules).
# Usage: bash scripts/gpu_pmc_prod.sh <tag> [extra bench.py args]
set -o pipefail
tag=${1:-prod}; shift
out=gpurun_out/pmc_$tag
mkdir -p $out
export TMPDIR=/tmp
rocprofv3 -L > $out/counters_list.txt 2>&1 || true
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE TA_TA_BUSY_sum TD_TD_BUSY_sum" \
            "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
            "FETCH_SIZE TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE" \
            "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_TAG_STALL_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctrs -d $out/p$i -o p --output-format csv -- python3 bench.py --steps 2 --warmup 1 "$@" > $out/b$i.json 2> $out/b$i.log || { echo "pass $i failed"; tail -5 $out/b$i.log; exit 1; }
  echo "pass $i done"
done
python3 scripts/pmc_summary.py $out "tl_fwd_multi|tl_t_multi" $out/summary.txt
find $out -name "*.csv" -size +20M -delete
head -80 $out/summary.txt
