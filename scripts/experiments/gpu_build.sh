#!/bin/bash
# Device-side from_labeled + device entity-id unique: GPU tests, then the construction profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_build.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu_build.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_build.log
timeout -k 10 600 python scripts/build_profile.py > gpurun_out/build_profile2.log 2>&1 || { echo "build profile failed"; tail -30 gpurun_out/build_profile2.log; exit 1; }
grep -E "built in|data " gpurun_out/build_profile2.log
grep -A14 "RE coordinate built" gpurun_out/build_profile2.log | tail -12 | cut -c1-160
