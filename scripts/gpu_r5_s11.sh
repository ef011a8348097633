#!/bin/bash
# Round 5 step 11: batched triangular solves instead of explicit inverses (row space): tests, cold profile, game5pl.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5s11
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_game_gpu.py -k "trsv or row_space or gram or materialize or game" -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
bash scripts/gpu_r5_cold.sh > $out/cold.log 2>&1 || { tail -20 $out/cold.log; exit 1; }
grep -E "^# window|seg_gram|nested|row-space batch|fused primal batch" $out/cold.log | head -8
timeout -k 10 400 python -u bench_game.py --config game5pl --steps 5 --warmup 2 > $out/g.json 2> $out/g.log || { echo "bench failed"; tail -30 $out/g.log; exit 1; }
echo "game5pl: $(grep -o '"coordinate_ms[^}]*}' $out/g.json) $(grep -o 'sweeps (ms).*' $out/g.log) $(grep -o '"cold_first_sweep_ms[^,]*' $out/g.json) $(grep -o '"ms_per_step[^,]*' $out/g.json)"
