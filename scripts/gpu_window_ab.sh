#!/bin/bash
# Window rounds (tiled.split_window / tl_stream_win): GPU parity tests, then the headline bench with and without
# window rounds (same binary, layout switch PML_TL_WINDOW), then the full GPU suite.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -k "window or narrow or multi or two_loop" > gpurun_out/pytest_window.log 2>&1 || { echo "window tests failed"; tail -40 gpurun_out/pytest_window.log; exit 1; }
tail -1 gpurun_out/pytest_window.log
for wnd in 1 0 1; do
  PML_TL_WINDOW=$wnd timeout -k 10 300 python bench.py --game off --steps 10 --warmup 3 > gpurun_out/bench_win$wnd.json 2> gpurun_out/bench_win$wnd.log || { echo "bench win=$wnd failed"; tail -20 gpurun_out/bench_win$wnd.log; exit 1; }
  echo "window=$wnd: $(cut -c1-200 gpurun_out/bench_win$wnd.json)"
done
bash scripts/gpu_full.sh
