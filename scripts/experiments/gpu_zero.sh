#!/bin/bash
# Zero-point evaluation from the offsets + reordered tolerance pass: tests, FE pass count, game5.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_zero.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_zero.log; exit 1; }
tail -1 gpurun_out/pytest_zero.log
timeout -k 10 600 python -u bench_game.py --config game5 --steps 3 --warmup 2 --log-level DEBUG > gpurun_out/zero_g5.json 2> gpurun_out/zero_g5.log || { echo "failed"; tail -20 gpurun_out/zero_g5.log; exit 1; }
grep -E "passes in the update|Update coordinate global" gpurun_out/zero_g5.log | tail -4 | cut -c1-160
cat gpurun_out/zero_g5.json | cut -c1-200
