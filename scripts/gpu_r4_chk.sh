#!/bin/bash
# Checkpoint: GAME / kernel GPU tests touching the lean kernel and the FE device path, game5pl bench.
set -o pipefail
mkdir -p gpurun_out/r4chk
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_game_gpu.py tests/test_kernels_gpu.py tests/test_bench_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4chk/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r4chk/pytest.log; exit 1; }
tail -2 gpurun_out/r4chk/pytest.log
timeout -k 10 400 python -u bench_game.py --config game5pl --steps 5 --warmup 2 > gpurun_out/r4chk/g.json 2> gpurun_out/r4chk/g.log || { echo "bench failed"; tail -30 gpurun_out/r4chk/g.log; exit 1; }
cut -c130-330 gpurun_out/r4chk/g.json; grep "sweeps (ms)" gpurun_out/r4chk/g.log
