#!/bin/bash
# Round 5: packed-triangle row-space TRON (variant 7) with per-K occupancy hints (ops/_lib/exp/libpml_glm_<v>.so).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5rstri2
mkdir -p $out
run() {  # name lib n
  PML_GLM_LIB=$2 timeout -k 10 300 python3 -u scripts/rs_tron_bench.py 1250000 $3 5,7 > $out/$1_n$3.log 2>&1 || { echo "$1 n=$3 failed"; tail -20 $out/$1_n$3.log; exit 1; }
  echo "== $1 n=$3"; grep -v amdgpu.ids $out/$1_n$3.log | grep -v ordered
}
L=photon_ml_amd/ops/_lib
run base $L/libpml_glm.so 20 && run w20 $L/exp/libpml_glm_w20.so 20 && run base $L/libpml_glm.so 24 && \
run w24 $L/exp/libpml_glm_w24.so 24 && run base $L/libpml_glm.so 32 && run w32 $L/exp/libpml_glm_w32.so 32
