#!/bin/bash
# 2-rank data-parallel + entity-sharded GAME rehearsal on ONE GPU (both ranks on cuda:0, gloo collectives) at the
# config-5 per-GPU shape (1.25M entities per rank): build (routing) time and sweep time.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
PML_DIST_BACKEND=gloo timeout -k 10 1000 python -u bench_game.py --gpus 2 --config game5 --steps 2 --warmup 1 --log-level INFO > gpurun_out/game5_2rank_gloo.json 2> gpurun_out/game5_2rank_gloo.log || { echo "rehearsal failed"; tail -40 gpurun_out/game5_2rank_gloo.log; exit 1; }
grep -E "route rows|coordinates built|data generated" gpurun_out/game5_2rank_gloo.log
cut -c1-400 gpurun_out/game5_2rank_gloo.json
