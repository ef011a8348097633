#!/bin/bash
# GLM passes per fixed-effect update (GAME config 5).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u bench_game.py --config game5 --steps 1 --warmup 2 --log-level DEBUG > gpurun_out/fepass.json 2> gpurun_out/fepass.log || { echo "failed"; tail -20 gpurun_out/fepass.log; exit 1; }
grep -E "passes in the update|Update coordinate global" gpurun_out/fepass.log | cut -c1-200
