#!/bin/bash
# Full check (output dir = $1): full GPU test suite, smoke, headline bench (+ game5pl bf16 / fp64 keys).
set -o pipefail
mkdir -p gpurun_out/${1:-r4full}
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${1:-r4full}/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${1:-r4full}/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/${1:-r4full}/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${1:-r4full}/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${1:-r4full}/smoke.log; exit 1; }
tail -1 gpurun_out/${1:-r4full}/smoke.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${1:-r4full}/bench.json 2> gpurun_out/${1:-r4full}/bench.log || { echo "bench failed"; tail -30 gpurun_out/${1:-r4full}/bench.log; exit 1; }
cat gpurun_out/${1:-r4full}/bench.json
