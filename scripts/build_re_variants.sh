#!/bin/bash
# Build A/B variants of the random-effect kernel library into ops/_lib/exp/ (CPU, hipcc cross-compile).
# usage: build_re_variants.sh NAME "DEFINES" [NAME "DEFINES" ...]
set -e
cd "$(dirname "$0")/.."
mkdir -p photon_ml_amd/ops/_lib/exp
while [ $# -ge 2 ]; do
  n=$1; d=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result $d \
    photon_ml_amd/ops/csrc/re_kernels.hip -o photon_ml_amd/ops/_lib/exp/libpml_re_$n.so &
done
wait
ls -la photon_ml_amd/ops/_lib/exp/
