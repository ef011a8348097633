#!/bin/bash
# Idle-gap attribution (GPU waiting on the host) in the GAME config-5 fixed-effect coordinate and the headline
# bench's timed window: rocprofv3 kernel + marker trace, scripts/prof_window.py gap tables.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
PML_TRACE=1 timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace -d $R/gpurun_out/prof_g5 -o prof -- python3 $R/bench_game.py --config game5 --steps 1 --warmup 2 > $R/gpurun_out/gaps_g5.json 2> $R/gpurun_out/gaps_g5.log || { echo "game prof failed"; tail -30 $R/gpurun_out/gaps_g5.log; exit 1; }
db=$(find $R/gpurun_out/prof_g5 -name "*.db" | head -1)
python3 $R/scripts/prof_window.py "$db" "Update coordinate global" $R/gpurun_out/game5_fe_window_gaps.md > /dev/null && cat $R/gpurun_out/game5_fe_window_gaps.md | tail -45
python3 $R/scripts/prof_window.py "$db" "Update coordinate per-entity" $R/gpurun_out/game5_re_window_gaps.md > /dev/null
rm -rf $R/gpurun_out/prof_g5
