#!/bin/bash
# Round 5: where the cold first sweep goes -- the RE solver-component build window (rocprofv3 kernel + marker trace).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
PML_TRACE=1 timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace -d $R/gpurun_out/prof_cold -o prof -- python3 $R/bench_game.py --config game5pl --steps 1 --warmup 1 --log-level DEBUG > $R/gpurun_out/prof_cold.json 2> $R/gpurun_out/prof_cold.log || { echo "prof failed"; tail -30 $R/gpurun_out/prof_cold.log; exit 1; }
db=$(find $R/gpurun_out/prof_cold -name "*.db" | head -1)
python3 $R/scripts/prof_window.py "$db" "solver components" $R/gpurun_out/cold_components_window.md > /dev/null && head -60 $R/gpurun_out/cold_components_window.md
grep -E "row-space batch|fused primal batch|solver components" $R/gpurun_out/prof_cold.log | cut -c1-160
rm -rf $R/gpurun_out/prof_cold
