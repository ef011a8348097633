#!/bin/bash
# XCD-aware transpose item order A/B on the headline bench (+ the bucketed-gradient bitwise test).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -k "bucketed or multi or transpose or tiled" > gpurun_out/pytest_xcd.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_xcd.log; exit 1; }
tail -1 gpurun_out/pytest_xcd.log
for x in 8 0 8; do
  PML_TL_XCD=$x timeout -k 10 900 python bench.py > gpurun_out/bench_xcd_$x.json 2> gpurun_out/bench_xcd_$x.log || { echo "bench $x failed"; tail -30 gpurun_out/bench_xcd_$x.log; exit 1; }
  echo "PML_TL_XCD=$x"; cat gpurun_out/bench_xcd_$x.json | cut -c1-230
done
