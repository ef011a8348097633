#!/bin/bash
# Timed-window kernel-busy profiles: headline bench (125M rows) and the GAME fixed-effect coordinate (game5).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
PML_TRACE=1 timeout -k 10 900 rocprofv3 --kernel-trace --marker-trace -d $R/gpurun_out/prof_win -o prof -- python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/prof_win.json 2> $R/gpurun_out/prof_win.log || { echo "bench prof failed"; tail -30 $R/gpurun_out/prof_win.log; exit 1; }
cat $R/gpurun_out/prof_win.json
db=$(find $R/gpurun_out/prof_win -name "*.db" | head -1)
python3 $R/scripts/prof_window.py "$db" "bench timed steps" $R/gpurun_out/bench_125M_timed_window.md > /dev/null && head -30 $R/gpurun_out/bench_125M_timed_window.md
rm -rf $R/gpurun_out/prof_win
PML_TRACE=1 timeout -k 10 900 rocprofv3 --kernel-trace --marker-trace -d $R/gpurun_out/prof_g5 -o prof -- python3 $R/bench_game.py --config game5 --steps 1 --warmup 2 > $R/gpurun_out/prof_g5.json 2> $R/gpurun_out/prof_g5.log || { echo "game prof failed"; tail -30 $R/gpurun_out/prof_g5.log; exit 1; }
db=$(find $R/gpurun_out/prof_g5 -name "*.db" | head -1)
python3 $R/scripts/prof_window.py "$db" "Update coordinate global" $R/gpurun_out/game5_fe_window.md > /dev/null && head -40 $R/gpurun_out/game5_fe_window.md
python3 $R/scripts/prof_window.py "$db" "Update coordinate per-entity" $R/gpurun_out/game5_re_window.md > /dev/null && head -30 $R/gpurun_out/game5_re_window.md
rm -rf $R/gpurun_out/prof_g5
cd /tmp
PML_TRACE=1 PML_TRON_STATS=1 timeout -k 10 900 rocprofv3 --kernel-trace --marker-trace -d $R/gpurun_out/prof_g5pl -o prof -- python3 $R/bench_game.py --config game5pl --steps 1 --warmup 2 > $R/gpurun_out/prof_g5pl.json 2> $R/gpurun_out/prof_g5pl.log || { echo "game5pl prof failed"; tail -30 $R/gpurun_out/prof_g5pl.log; exit 1; }
db=$(find $R/gpurun_out/prof_g5pl -name "*.db" | head -1)
python3 $R/scripts/prof_window.py "$db" "primal block-diagonal solve" $R/gpurun_out/game5pl_primal_window.md > /dev/null && head -40 $R/gpurun_out/game5pl_primal_window.md
rm -rf $R/gpurun_out/prof_g5pl
grep -E "entity-masked|block-diagonal TRON" $R/gpurun_out/prof_g5pl.log || true
