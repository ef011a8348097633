#!/bin/bash
# Round 5: row-space / primal split for n in (64, 192] (PML_RS_BIG_NNZ_RATIO) on game5pl.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5ratio
mkdir -p $out
for r in ${RATIOS:-0.6 0.45 0.35 0.8}; do
  PML_RS_BIG_NNZ_RATIO=$r timeout -k 10 400 python -u bench_game.py --config game5pl --steps 5 --warmup 2 > $out/g$r.json 2> $out/g$r.log || { echo "bench failed"; tail -30 $out/g$r.log; exit 1; }
  echo "ratio=$r: $(grep -o '"coordinate_ms[^}]*}' $out/g$r.json) $(grep -o 'sweeps (ms).*' $out/g$r.log) $(grep -o '"cold_first_sweep_ms[^,]*' $out/g$r.json)"
done
