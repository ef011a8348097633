#!/bin/bash
# BASELINE configs 3 (OWL-QN, L1, 10M features) and 4 (Poisson TRON) with the current kernels, plus TCC counters
# of the OWL-QN forward / transpose kernels (L2 behaviour of the 40 MB coefficient vector).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r3}
for cfg in owlqn tron; do
  timeout -k 10 600 python bench.py --config $cfg --game off > gpurun_out/bench_${cfg}_$tag.json 2> gpurun_out/bench_${cfg}_$tag.log || { echo "$cfg failed"; tail -20 gpurun_out/bench_${cfg}_$tag.log; exit 1; }
  cut -c1-330 gpurun_out/bench_${cfg}_$tag.json
done
out=gpurun_out/pmc_owlqn_$tag
mkdir -p $out
i=0
for ctrs in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE" "TA_TA_BUSY_sum TD_TD_BUSY_sum SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctrs -d $out/p$i -o p --output-format csv -- python3 bench.py --config owlqn --game off --steps 2 --warmup 1 > $out/b$i.json 2> $out/b$i.log || { echo "pmc pass $i failed"; tail -5 $out/b$i.log; exit 1; }
done
python3 scripts/pmc_summary.py $out "tl_fwd_multi|tl_t_multi" $out/summary.txt
find $out -name "*.csv" -size +20M -delete
cat $out/summary.txt
