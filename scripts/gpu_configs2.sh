#!/bin/bash
# BASELINE configs 3 (OWL-QN L1, 10M features) and 4 (Poisson TRON) at their per-GPU shapes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python bench.py --config owlqn --steps 5 --warmup 2 > gpurun_out/owlqn.json 2> gpurun_out/owlqn.log || { echo "owlqn failed"; tail -30 gpurun_out/owlqn.log; exit 1; }
cat gpurun_out/owlqn.json
timeout -k 10 900 python bench.py --config tron --steps 3 --warmup 1 > gpurun_out/tron.json 2> gpurun_out/tron.log || { echo "tron failed"; tail -30 gpurun_out/tron.log; exit 1; }
cat gpurun_out/tron.json
