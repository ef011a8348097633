#!/bin/bash
# GAME: new GPU tests (sampling, device RE build), then both config-5 presets of bench_game.py.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_sampling.py tests/test_game_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_game2.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_game2.log; exit 1; }
tail -2 gpurun_out/pytest_game2.log
for cfg in game5 game5pl; do
  timeout -k 10 900 python -u bench_game.py --config $cfg --steps 3 --warmup 3 > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.log || { echo "bench $cfg failed"; tail -30 gpurun_out/bench_$cfg.log; exit 1; }
  grep -E "built in|generated in|iteration|final" gpurun_out/bench_$cfg.log | tail -12
  cat gpurun_out/bench_$cfg.json
done
