#!/bin/bash
# Round 6 step 23: HBM bytes of the game5pl fp64 sweep's dominant kernels (lean RE TRON, FE TL passes, row-space
# TRON, back-map): FETCH_SIZE per dispatch -> achieved bandwidth vs the kernels' durations.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6s23
mkdir -p $out
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-include-regex "re_tron_lean|tl_fwd_multi|tl_t_multi|rs_tron|rs_primal|btrsv" -d $out/p1 -o p --output-format csv -- python3 $R/bench_game.py --config game5pl --precision f64 --steps 1 --warmup 1 > $out/b1.log 2>&1 || { echo "pmc pass failed"; tail -5 $out/b1.log; exit 1; }
python3 $R/scripts/pmc_summary.py $out "re_tron_lean|tl_fwd_multi|tl_t_multi|rs_tron|rs_primal|btrsv" $out/summary.txt
find $out -name "*.csv" -delete
cat $out/summary.txt
