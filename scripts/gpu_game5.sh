#!/bin/bash
# Device-side RE dataset build + device-resident RE models: GAME GPU tests, small preset, BASELINE config 5 preset.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python __graft_entry__.py build > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_game_gpu.py -x -q > gpurun_out/pytest_game.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_game.log; exit 1; }
tail -1 gpurun_out/pytest_game.log
timeout -k 10 600 python bench_game.py --steps 3 --warmup 1 > gpurun_out/bench_game_small.json 2> gpurun_out/bench_game_small.err || { echo "small failed"; tail -20 gpurun_out/bench_game_small.err; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_game_small.err | tail -6; cat gpurun_out/bench_game_small.json
timeout -k 10 1000 python bench_game.py --config game5 --steps 2 --warmup 1 > gpurun_out/bench_game5.json 2> gpurun_out/bench_game5.err || { echo "game5 failed"; tail -20 gpurun_out/bench_game5.err; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_game5.err | tail -8; cat gpurun_out/bench_game5.json
