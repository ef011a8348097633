#!/bin/bash
# Round 5: which entities go to the register-resident cluster kernel (PML_RE_RES_TAIL_SHARE: more than 1/share of
# the fused batch's non-zeros) on game5pl. Lean launch alone is 35.2 ms with the largest entities on one workgroup.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5tail
mkdir -p $out
for t in ${SHARES:-256 1024 4096 16384}; do
  PML_RE_RES_TAIL_SHARE=$t timeout -k 10 400 python -u bench_game.py --config game5pl --steps 5 --warmup 2 --log-level INFO > $out/g$t.json 2> $out/g$t.log || { echo "bench failed"; tail -30 $out/g$t.log; exit 1; }
  echo "share=$t: $(grep -o '"coordinate_ms[^}]*}' $out/g$t.json) $(grep -o 'sweeps (ms).*' $out/g$t.log) $(grep -o '"cold_first_sweep_ms[^,]*' $out/g$t.json)"
  grep -o "'resident': {[^}]*}" $out/g$t.log | head -1
done
