#!/bin/bash
# Round 5: row-space TRON, packed-triangle LDS (variant 7) vs the padded layout (variant 5), 1.25M problems.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5rstri
mkdir -p $out
for n in ${NS:-32 24 20}; do
  timeout -k 10 300 python3 -u scripts/rs_tron_bench.py 1250000 $n 5,7 > $out/n$n.log 2>&1 || { echo "n=$n failed"; tail -20 $out/n$n.log; exit 1; }
  echo "== n=$n"; grep -v amdgpu.ids $out/n$n.log
done
