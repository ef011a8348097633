#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --rows-per-gpu 16000000 --steps 5 --warmup 1 > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.log || { tail -30 gpurun_out/prof/bench.log; exit 1; }
find gpurun_out/prof -name "*stats*" | head
