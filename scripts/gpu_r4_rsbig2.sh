#!/bin/bash
# RE window of game5pl at PML_RS_NMAX 64 vs 128 (rs_tron_big_kernel vs primal fused kernel).
set -o pipefail
for nm in 64 128; do
  PML_RS_NMAX=$nm bash scripts/gpu_r4_window.sh game5pl g5pl_rs$nm || exit 1
done
