#!/bin/bash
# Round 5 step 16: lean kernel with one row group per function-evaluation batch (LEAN_UF=1): RE tests, game5pl.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5s16
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_game_gpu.py tests/test_fastpath_parity_gpu.py -k "lean or fused or game or entity" -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 400 python -u bench_game.py --config game5pl --steps 5 --warmup 2 > $out/g.json 2> $out/g.log || { echo "bench failed"; tail -30 $out/g.log; exit 1; }
echo "game5pl: $(grep -o '"coordinate_ms[^}]*}' $out/g.json) $(grep -o 'sweeps (ms).*' $out/g.log) $(grep -o '"cold_first_sweep_ms[^,]*' $out/g.json)"
