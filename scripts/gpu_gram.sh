#!/bin/bash
# Vector-free two-loop for long device vectors: A/B on the headline bench and GAME config 5.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for g in 1000000000000 262144; do
PML_LBFGS_GRAM_MIN_DIM=$g timeout -k 10 600 python bench.py > gpurun_out/gram_b$g.json 2> gpurun_out/gram_b$g.log || { echo "bench $g failed"; tail -30 gpurun_out/gram_b$g.log; exit 1; }
echo "gram_min=$g"; cat gpurun_out/gram_b$g.json; grep -h final gpurun_out/gram_b$g.log
done
for g in 1000000000000 262144; do
PML_LBFGS_GRAM_MIN_DIM=$g timeout -k 10 600 python bench_game.py --config game5 --steps 5 > gpurun_out/gram_g$g.json 2> gpurun_out/gram_g$g.log || { echo "game $g failed"; tail -30 gpurun_out/gram_g$g.log; exit 1; }
echo "gram_min=$g"; cat gpurun_out/gram_g$g.json; grep -h "coordinate global\|final" gpurun_out/gram_g$g.log | tail -4
done
