#!/bin/bash
# RE / FE coordinate and model-materialisation windows of a GAME preset (rocprofv3 kernel + marker trace)
# -> gpurun_out/<TAG>_{re,fe,materialize}_window.md
# usage: gpu_r4_window.sh PRESET TAG [extra bench_game args]
set -o pipefail
P=$1; TAG=$2; shift 2
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
PML_TRACE=1 timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace -d $R/gpurun_out/prof_$TAG -o prof -- python3 $R/bench_game.py --config $P --steps 1 --warmup 2 "$@" > $R/gpurun_out/prof_$TAG.json 2> $R/gpurun_out/prof_$TAG.log || { echo "$P prof failed"; tail -30 $R/gpurun_out/prof_$TAG.log; exit 1; }
db=$(find $R/gpurun_out/prof_$TAG -name "*.db" | head -1)
python3 $R/scripts/prof_window.py "$db" "Update coordinate per-entity" $R/gpurun_out/${TAG}_re_window.md > /dev/null && head -16 $R/gpurun_out/${TAG}_re_window.md
python3 $R/scripts/prof_window.py "$db" "Update coordinate global" $R/gpurun_out/${TAG}_fe_window.md > /dev/null && head -8 $R/gpurun_out/${TAG}_fe_window.md
python3 $R/scripts/prof_window.py "$db" "materialize model" $R/gpurun_out/${TAG}_materialize_window.md > /dev/null && head -14 $R/gpurun_out/${TAG}_materialize_window.md
rm -rf $R/gpurun_out/prof_$TAG
