#!/bin/bash
# Round 5 step 12: block layout for the K = 48 row-space class: rs tests, game5pl + RE window.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5s12
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "rs_tron or row_space" -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" $out/pytest.log | tail -30; tail -40 $out/pytest.log; exit 1; }
grep -cE "PASSED" $out/pytest.log; tail -1 $out/pytest.log
for n in; do
  timeout -k 10 300 python3 -u scripts/rs_tron_bench.py 1250000 $n 4,5 > $out/rs_n$n.log 2>&1 || { echo "n=$n failed"; tail -20 $out/rs_n$n.log; exit 1; }
  echo "== n=$n"; grep -v amdgpu.ids $out/rs_n$n.log | grep -v ordered
done
timeout -k 10 400 python -u bench_game.py --config game5pl --steps 5 --warmup 2 > $out/g.json 2> $out/g.log || { echo "bench failed"; tail -30 $out/g.log; exit 1; }
echo "game5pl: $(grep -o '"coordinate_ms[^}]*}' $out/g.json) $(grep -o 'sweeps (ms).*' $out/g.log) $(grep -o '"cold_first_sweep_ms[^,]*' $out/g.json)"
bash scripts/gpu_r4_window.sh game5pl r5s12 > $out/window.log 2>&1 || { tail -20 $out/window.log; exit 1; }
grep -A12 "per-entity" $out/window.log | head -14
