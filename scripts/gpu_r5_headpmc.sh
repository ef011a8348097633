#!/bin/bash
# Round 5: PMC of the headline kernels at the production shape (125M rows x 1M features x 100 nnz, bf16) with the
# dispatch durations (effective clock) — the TA-floor note (profiles/headline_floor_r5.md).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5headpmc
mkdir -p $out
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE TA_TA_BUSY_sum TD_TD_BUSY_sum" \
            "FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctrs -d $out/p$i -o p --output-format csv -- python3 bench.py --steps 2 --warmup 1 --game off > $out/b$i.json 2> $out/b$i.log || { echo "pass $i failed"; tail -5 $out/b$i.log; exit 1; }
done
python3 scripts/pmc_summary.py $out "tl_fwd_multi|tl_t_multi" $out/summary.txt > /dev/null
find $out -name "*.csv" -delete
cat $out/summary.txt
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --game off > $out/bench.json 2> $out/bench.log || { echo "bench failed"; tail -5 $out/bench.log; exit 1; }
cat $out/bench.json
