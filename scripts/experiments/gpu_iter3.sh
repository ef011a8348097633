#!/bin/bash
# Random-projection GPU test + TL ablations.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_game_gpu.py -x -q --timeout 200 --timeout-method thread -k "random_projection or mfma or scoring" > gpurun_out/pytest_rp.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_rp.log; exit 1; }
tail -2 gpurun_out/pytest_rp.log
bash scripts/gpu_ablate.sh
