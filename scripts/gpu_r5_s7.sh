#!/bin/bash
# Round 5 step 7: RE kernel/game GPU tests with the prefetch + 4-wide-gather lean kernel, then game5pl (bench_game,
# 5 timed sweeps) and the RE window.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5s7
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_game_gpu.py tests/test_fastpath_parity_gpu.py -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" $out/pytest.log | tail -30; tail -40 $out/pytest.log; exit 1; }
grep -cE "PASSED" $out/pytest.log; tail -2 $out/pytest.log
timeout -k 10 400 python -u bench_game.py --config game5pl --steps 5 --warmup 2 > $out/g.json 2> $out/g.log || { echo "bench failed"; tail -30 $out/g.log; exit 1; }
echo "game5pl: $(grep -o '"coordinate_ms[^}]*}' $out/g.json) $(grep -o 'sweeps (ms).*' $out/g.log) $(grep -o '"cold_first_sweep_ms[^,]*' $out/g.json)"
bash scripts/gpu_r4_window.sh game5pl r5s7 || exit 1
