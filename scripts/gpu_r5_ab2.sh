#!/bin/bash
# Round 5: lean RE kernel A/B (row-pointer prefetch + global-space loads + 4-wide LDS gathers) on the
# 43K-entity micro, strided (QUAD=0) and quad-padded (QUAD=1) rows. -> gpurun_out/r5ab2/
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5ab2
mkdir -p $out
for v in ${@:-old new}; do
  for q in ${QS:-0 1}; do
    PML_BENCH_QUAD=$q PML_RE_LIB=photon_ml_amd/ops/_lib/exp/libpml_re_$v.so timeout -k 10 240 \
      python3 -u scripts/re_fused_bench.py 43000 lean > $out/$v.q$q.log 2>&1 || { echo "$v q$q failed"; tail -20 $out/$v.q$q.log; exit 1; }
    echo "== $v quad=$q"; grep -v amdgpu.ids $out/$v.q$q.log | tail -2
  done
done
