#!/bin/bash
# Where a whole timed GAME run goes (config-5 preset, 3 timed sweeps + the model materialisation): rocprofv3 kernel
# + marker trace, scripts/prof_window.py tables of the "timed sweeps" and "materialize model" regions.
set -o pipefail
R=$GRAFT_REPO_ROOT
cfg=${1:-game5}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
PML_TRACE=1 timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace -d $R/gpurun_out/prof_sw -o prof -- python3 $R/bench_game.py --config $cfg --steps 3 --warmup 2 > $R/gpurun_out/sweep_$cfg.json 2> $R/gpurun_out/sweep_$cfg.log || { echo "prof failed"; tail -30 $R/gpurun_out/sweep_$cfg.log; exit 1; }
db=$(find $R/gpurun_out/prof_sw -name "*.db" | head -1)
python3 $R/scripts/prof_window.py "$db" "timed sweeps" $R/gpurun_out/${cfg}_timed_window.md > /dev/null && head -60 $R/gpurun_out/${cfg}_timed_window.md
python3 $R/scripts/prof_window.py "$db" "materialize model" $R/gpurun_out/${cfg}_materialize_window.md > /dev/null && head -20 $R/gpurun_out/${cfg}_materialize_window.md
rm -rf $R/gpurun_out/prof_sw
