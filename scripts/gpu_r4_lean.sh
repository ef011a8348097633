#!/bin/bash
# Streaming RE kernel A/B on the game5pl-like microbenchmark: in-tree (stream + lean at 4 waves/SIMD), lean at
# 3 waves/SIMD (w3a: U 1/2, w3b: U 1/3), stream with 2 / 4 row groups per wave batch (s2, s4).
set -o pipefail
mkdir -p gpurun_out/r4lean2
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/re_fused_bench.py 43000 stream,lean > gpurun_out/r4lean2/a.log 2>&1 || { echo "a failed"; tail -20 gpurun_out/r4lean2/a.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4lean2/a.log
for v in w3a:lean w3b:lean s2:stream s4:stream; do
  n=${v%%:*}; k=${v##*:}
  PML_RE_LIB=photon_ml_amd/ops/_lib/exp/libpml_re_$n.so timeout -k 10 300 python -u scripts/re_fused_bench.py 43000 $k > gpurun_out/r4lean2/$n.log 2>&1 || { echo "$n failed"; tail -20 gpurun_out/r4lean2/$n.log; exit 1; }
  echo "variant $n:"; grep -v amdgpu.ids gpurun_out/r4lean2/$n.log | tail -1
done
