#!/bin/bash
# End-of-session check: the whole GPU suite, smoke(), and the driver's default bench.py (headline + game5pl).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_final.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_final.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { tail -20 gpurun_out/smoke_final.log; exit 1; }
tail -1 gpurun_out/smoke_final.log
timeout -k 10 400 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.log || { tail -20 gpurun_out/bench_final.log; exit 1; }
cut -c1-400 gpurun_out/bench_final.json
