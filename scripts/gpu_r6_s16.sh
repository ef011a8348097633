#!/bin/bash
# Round 6 step 16: gated finish with its readback queued ahead (A/B + window), then the RE tail-share A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash scripts/gpu_r6_s14.sh && bash scripts/gpu_r6_s15.sh
