#!/bin/bash
# 2-rank entity-sharded GAME rehearsal on one GPU (config-5 shape per rank), BASELINE configs 3/4, MFMA Hessian path.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_rehearsal.sh && bash scripts/gpu_cfg34.sh r3 && bash scripts/gpu_hess.sh
