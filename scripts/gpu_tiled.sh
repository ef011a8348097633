#!/bin/bash
# Tiled-layout validation: kernel parity tests, microbench tiled vs segmented, full bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python __graft_entry__.py build > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/pytest_kernels.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_kernels.log; exit 1; }
tail -3 gpurun_out/pytest_kernels.log
timeout -k 10 300 python scripts/kbench.py --rows 16000000 --layout tiled --configs "0,0,0" > gpurun_out/kbench_tiled.log 2>&1 || { echo "kbench tiled failed"; tail -30 gpurun_out/kbench_tiled.log; exit 1; }
tail -3 gpurun_out/kbench_tiled.log
timeout -k 10 300 python scripts/kbench.py --rows 16000000 --layout segmented --configs "0,0,0" > gpurun_out/kbench_seg.log 2>&1 || { echo "kbench seg failed"; tail -30 gpurun_out/kbench_seg.log; exit 1; }
tail -3 gpurun_out/kbench_seg.log
timeout -k 10 900 python bench.py > gpurun_out/bench_tiled.json 2> gpurun_out/bench_tiled.log || { echo "bench failed"; tail -40 gpurun_out/bench_tiled.log; exit 1; }
cat gpurun_out/bench_tiled.json
tail -4 gpurun_out/bench_tiled.log
