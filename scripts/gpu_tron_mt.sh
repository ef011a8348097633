#!/bin/bash
# TRON margin-space trial: device tests, then the TRON bench config with the trial path off / on.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_game_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "tron_margin or scoring_on_device or margin_space" > gpurun_out/pytest_tmt.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_tmt.log; exit 1; }
grep -c PASSED gpurun_out/pytest_tmt.log; tail -1 gpurun_out/pytest_tmt.log
for m in 0 1; do
PML_TRON_MARGIN_TRIAL=$m timeout -k 10 600 python bench.py --config tron --steps 3 --warmup 1 > gpurun_out/tron_mt$m.json 2> gpurun_out/tron_mt$m.log || { echo "bench $m failed"; tail -30 gpurun_out/tron_mt$m.log; exit 1; }
echo "mt=$m"; cat gpurun_out/tron_mt$m.json; grep -h final gpurun_out/tron_mt$m.log
done
