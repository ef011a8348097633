#!/bin/bash
# BASELINE.json configs 3 and 4 at their per-GPU shapes (1 GPU).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python __graft_entry__.py build > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 900 python bench.py --config tron --steps 3 --warmup 1 > gpurun_out/bench_tron.json 2> gpurun_out/bench_tron.err || { echo "tron failed"; tail -20 gpurun_out/bench_tron.err; exit 1; }
cat gpurun_out/bench_tron.json
timeout -k 10 900 python bench.py --config owlqn --steps 5 --warmup 2 > gpurun_out/bench_owlqn.json 2> gpurun_out/bench_owlqn.err || { echo "owlqn failed"; tail -20 gpurun_out/bench_owlqn.err; exit 1; }
cat gpurun_out/bench_owlqn.json
