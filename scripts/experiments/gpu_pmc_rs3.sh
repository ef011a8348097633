#!/bin/bash
# PMC pass over rs_tron variants 2 / 3 at n = 16 and 20 (instruction mix, busy and wait cycles).
set -o pipefail
out=gpurun_out/pmc_rs3
mkdir -p $out
export TMPDIR=/tmp
for n in 16 20; do
  timeout -k 10 150 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $out/n$n -o p --output-format csv -- python3 scripts/rs_tron_bench.py 1250000 $n 2,3 > $out/rs_n$n.log 2>&1 || { echo "pass $n failed"; tail -5 $out/rs_n$n.log; exit 1; }
  python scripts/pmc_summary.py $out/n$n "rs_tron" $out/summary_n$n.txt > /dev/null
  echo "== n=$n"; cat $out/summary_n$n.txt
done
find $out -name "*.csv" -size +5M -delete
