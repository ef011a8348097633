#!/bin/bash
# Round-3 measurement set: full bench.py (GLM headline + driver-timed game5pl extra), game5 (uniform), and a
# kernel-trace window of the game5pl random-effect update.
# Usage: bash scripts/gpu_r3.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
tag=${1:-r3}
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd $R
t0=$(date +%s.%N); timeout -k 10 600 python bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.log || { echo "bench failed"; tail -30 gpurun_out/bench_$tag.log; exit 1; }
echo "bench wall $(echo "$(date +%s.%N) - $t0" | bc) s"; cut -c1-1200 gpurun_out/bench_$tag.json
timeout -k 10 600 python -u bench_game.py --config game5 --steps 3 --warmup 2 > gpurun_out/game5_$tag.json 2> gpurun_out/game5_$tag.log || { echo "game5 failed"; tail -30 gpurun_out/game5_$tag.log; exit 1; }
cut -c1-260 gpurun_out/game5_$tag.json
cd /tmp
PML_TRACE=1 timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace -d $R/gpurun_out/prof_g5pl -o prof -- python3 $R/bench_game.py --config game5pl --steps 1 --warmup 2 > $R/gpurun_out/prof_g5pl.json 2> $R/gpurun_out/prof_g5pl.log || { echo "game5pl prof failed"; tail -30 $R/gpurun_out/prof_g5pl.log; exit 1; }
db=$(find $R/gpurun_out/prof_g5pl -name "*.db" | head -1)
python3 $R/scripts/prof_window.py "$db" "Update coordinate per-entity" $R/gpurun_out/game5pl_re_window_$tag.md > /dev/null && head -30 $R/gpurun_out/game5pl_re_window_$tag.md
python3 $R/scripts/prof_window.py "$db" "Update coordinate global" $R/gpurun_out/game5pl_fe_window_$tag.md > /dev/null && head -24 $R/gpurun_out/game5pl_fe_window_$tag.md
rm -rf $R/gpurun_out/prof_g5pl
