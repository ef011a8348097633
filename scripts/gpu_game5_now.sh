#!/bin/bash
# GAME config-5 bench (1.25M entities x 1001 coefficients / GPU) with a per-phase JSON timeline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/g5_timeline.jsonl
PML_TIMELINE=$GRAFT_REPO_ROOT/gpurun_out/g5_timeline.jsonl timeout -k 10 900 python bench_game.py --config game5 --steps 2 --warmup 1 > gpurun_out/g5.json 2> gpurun_out/g5.log || { echo "game5 failed"; tail -30 gpurun_out/g5.log; exit 1; }
cat gpurun_out/g5.json
grep -v amdgpu.ids gpurun_out/g5.log | tail -8
