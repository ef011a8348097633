#!/bin/bash
# Round 4 checkpoint: full GPU test suite, headline bench (+ game5pl bf16 / fp64 keys), game5tall sweep.
set -o pipefail
mkdir -p gpurun_out/r4full
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4full/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r4full/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r4full/pytest_gpu.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4full/bench.json 2> gpurun_out/r4full/bench.log || { echo "bench failed"; tail -30 gpurun_out/r4full/bench.log; exit 1; }
cat gpurun_out/r4full/bench.json
timeout -k 10 300 python -u bench_game.py --config game5tall --steps 3 --warmup 2 > gpurun_out/r4full/game5tall.json 2> gpurun_out/r4full/game5tall.log || { echo "game5tall failed"; tail -30 gpurun_out/r4full/game5tall.log; exit 1; }
cut -c1-400 gpurun_out/r4full/game5tall.json
