#!/bin/bash
# game5pl random-effect coordinate window (rocprofv3 kernel + marker trace): the fused per-entity primal TRON,
# the row-space TRON and the rest of "Update coordinate per-entity".
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
PML_TRACE=1 timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace -d $R/gpurun_out/prof_g5pl -o prof -- python3 $R/bench_game.py --config game5pl --steps 1 --warmup 2 > $R/gpurun_out/prof_g5pl.json 2> $R/gpurun_out/prof_g5pl.log || { echo "game5pl prof failed"; tail -30 $R/gpurun_out/prof_g5pl.log; exit 1; }
db=$(find $R/gpurun_out/prof_g5pl -name "*.db" | head -1)
python3 $R/scripts/prof_window.py "$db" "Update coordinate per-entity" $R/gpurun_out/game5pl_re_window_r3f.md > /dev/null && head -30 $R/gpurun_out/game5pl_re_window_r3f.md
python3 $R/scripts/prof_window.py "$db" "Update coordinate global" $R/gpurun_out/game5pl_fe_window_r3f.md > /dev/null && head -12 $R/gpurun_out/game5pl_fe_window_r3f.md
rm -rf $R/gpurun_out/prof_g5pl
