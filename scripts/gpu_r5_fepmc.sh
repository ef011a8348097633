#!/bin/bash
# Round 5: PMC of the fixed-effect TL kernels on the game5pl shard, bf16 vs fp64 feature storage (what the extra
# fp64 time sits on: TA / TD / HBM / occupancy). One rocprofv3 run per counter pass and precision.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5fepmc
mkdir -p $out
for prec in bf16 f64; do
  i=0
  for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE TA_TA_BUSY_sum TD_TD_BUSY_sum" \
              "FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE TCP_TCC_READ_REQ_sum" \
              "SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctrs -d $out/${prec}_p$i -o p --output-format csv -- python3 bench_game.py --config game5pl --steps 1 --warmup 1 --precision $prec > $out/${prec}_b$i.json 2> $out/${prec}_b$i.log || { echo "$prec pass $i failed"; tail -5 $out/${prec}_b$i.log; exit 1; }
  done
  python3 scripts/pmc_summary.py $out/${prec}_p1 "tl_fwd_multi|tl_t_multi" $out/${prec}_s1.txt > /dev/null
  python3 scripts/pmc_summary.py $out/${prec}_p2 "tl_fwd_multi|tl_t_multi" $out/${prec}_s2.txt > /dev/null
  python3 scripts/pmc_summary.py $out/${prec}_p3 "tl_fwd_multi|tl_t_multi" $out/${prec}_s3.txt > /dev/null
  cat $out/${prec}_s?.txt > $out/summary_$prec.txt
done
find $out -name "*.csv" -delete
cat $out/summary_bf16.txt $out/summary_f64.txt
