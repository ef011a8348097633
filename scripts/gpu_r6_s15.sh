#!/bin/bash
# Round 6 step 15: RE tail-entity threshold A/B (register-resident workgroup clusters for more of the largest entities).
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6s15
mkdir -p $out
cd $R
for share in 256 1024 4096 256; do
  PML_RE_RES_TAIL_SHARE=$share timeout -k 10 300 python -u bench_game.py --config game5pl --steps 8 --warmup 3 --precision bf16 > $out/bench_s$share.json 2> $out/bench_s$share.log || { echo "bench $share failed"; tail -30 $out/bench_s$share.log; exit 1; }
  python3 -c "import json; d=json.load(open('$out/bench_s$share.json')); print('tail share $share', round(d['ms_per_step'],2), round(d['sweep_ms_median'],2), {k: round(v,2) for k,v in d['coordinate_ms'].items()}, d['cold_first_sweep_coordinate_ms'])"
  grep "RE solver routing" $out/bench_s$share.log | sed 's/.*routing/routing/'
done
