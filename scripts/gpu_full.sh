#!/bin/bash
# Full GPU test suite + smoke (what the driver runs at round end).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_full.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu_full.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
