#!/bin/bash
# Re-entry verification: full GPU suite + smoke, the headline bench (with its game5pl keys), and both GAME config-5
# presets with fp64 fixed-effect features (BASELINE precision) next to the bf16 default.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_full.sh || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench_verify.json 2> gpurun_out/bench_verify.log || { echo "bench failed"; tail -30 gpurun_out/bench_verify.log; exit 1; }
cut -c1-300 gpurun_out/bench_verify.json
for cfg in game5 game5pl; do
  timeout -k 10 600 python -u bench_game.py --config $cfg --precision f64 --steps 3 --warmup 2 > gpurun_out/${cfg}_f64.json 2> gpurun_out/${cfg}_f64.log || { echo "$cfg f64 failed"; tail -30 gpurun_out/${cfg}_f64.log; exit 1; }
  grep -E "data generated|built in|passes" gpurun_out/${cfg}_f64.log | tail -3
  cut -c1-400 gpurun_out/${cfg}_f64.json
done
