#!/bin/bash
# FE epilogue fusions: GLM / GAME GPU tests, torch-call attribution of a GAME sweep, game5pl bench.
set -o pipefail
out=gpurun_out/${1:-fefuse}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_game_gpu.py tests/test_bench_gpu.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 400 python -u scripts/fe_torch_calls.py game5pl $out/fe_calls.txt > $out/calls.log 2>&1 || { echo "calls failed"; tail -20 $out/calls.log; exit 1; }
timeout -k 10 400 python -u bench_game.py --config game5pl --steps 5 --warmup 2 > $out/g.json 2> $out/g.log || { echo "bench failed"; tail -30 $out/g.log; exit 1; }
cut -c1-600 $out/g.json; grep "sweeps (ms)" $out/g.log
