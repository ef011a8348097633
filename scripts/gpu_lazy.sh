#!/bin/bash
# Lazy row-space primal model + gram kernels: GPU tests (game, kernels), GAME config 5 lazy on / off.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_game_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_lazy.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_lazy.log; exit 1; }
tail -1 gpurun_out/pytest_lazy.log
for m in 1 0; do
PML_RE_LAZY_PRIMAL=$m timeout -k 10 600 python bench_game.py --config game5 --steps 5 > gpurun_out/lazy_g$m.json 2> gpurun_out/lazy_g$m.log || { echo "game $m failed"; tail -30 gpurun_out/lazy_g$m.log; exit 1; }
echo "lazy=$m"; cat gpurun_out/lazy_g$m.json; grep -h "coordinate\|final" gpurun_out/lazy_g$m.log | tail -11
done
