#!/bin/bash
set -o pipefail
rm -f gpurun_out/g5s_tl.jsonl
mkdir -p gpurun_out
export TMPDIR=/tmp
PML_TIMELINE=$GRAFT_REPO_ROOT/gpurun_out/g5s_tl.jsonl timeout -k 10 900 python bench_game.py --config game5 --steps 5 --warmup 3 > gpurun_out/g5s.json 2> gpurun_out/g5s.log || { echo "game5 failed"; tail -30 gpurun_out/g5s.log; exit 1; }
cat gpurun_out/g5s.json
grep -v amdgpu.ids gpurun_out/g5s.log | tail -9
