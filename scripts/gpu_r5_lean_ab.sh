#!/bin/bash
# Round 5: vectorised quad row pass A/B of the lean streaming RE kernel (43K game5pl-like entities).
# Variants: ops/_lib/exp/libpml_re_<v>.so (scripts/build_re_variants.sh). -> gpurun_out/r5leanab/
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5leanab
mkdir -p $out
for v in ${@:-old v3 v4a v4b v4c}; do
  PML_RE_LIB=photon_ml_amd/ops/_lib/exp/libpml_re_$v.so timeout -k 10 240 python3 -u scripts/re_fused_bench.py 43000 stream,lean > $out/$v.log 2>&1 || { echo "$v failed"; tail -20 $out/$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $out/$v.log | tail -3
done
