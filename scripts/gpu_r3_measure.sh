#!/bin/bash
# Round-3 measurements: GAME config 5 (uniform and power-law entity sizes) with bf16 and fp64 fixed-effect
# features, then BASELINE configs 3 / 4 and the OWL-QN PMC passes (scripts/gpu_cfg34.sh).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r3m}
for cfg in game5 game5pl; do
  for prec in bf16 f64; do
    timeout -k 10 400 python -u bench_game.py --config $cfg --precision $prec --steps 3 --warmup 2 --log-level INFO \
      > gpurun_out/${cfg}_${prec}_$tag.json 2> gpurun_out/${cfg}_${prec}_$tag.log \
      || { echo "$cfg $prec failed"; tail -20 gpurun_out/${cfg}_${prec}_$tag.log; exit 1; }
    cut -c1-400 gpurun_out/${cfg}_${prec}_$tag.json
  done
done
bash scripts/gpu_cfg34.sh $tag
