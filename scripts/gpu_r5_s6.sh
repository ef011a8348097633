#!/bin/bash
# Round 5 step 6: lean kernel on rows padded to quads (row_pass_q) vs the strided pass (micro), the RE GPU tests,
# then game5pl (bench_game, 5 timed sweeps) and the RE window.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5s6
mkdir -p $out
for q in 1 0 1; do
  PML_BENCH_QUAD=$q timeout -k 10 240 python3 -u scripts/re_fused_bench.py 43000 lean > $out/micro_q$q.log 2>&1 || { echo "micro q=$q failed"; tail -20 $out/micro_q$q.log; exit 1; }
  echo "quad=$q: $(grep -v amdgpu.ids $out/micro_q$q.log | tail -1)"
done
timeout -k 10 900 python -u -m pytest tests/test_game_gpu.py tests/test_fastpath_parity_gpu.py -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; grep -E "PASS|FAIL|Error|error" $out/pytest.log | tail -30; tail -40 $out/pytest.log; exit 1; }
grep -cE "PASSED" $out/pytest.log; tail -2 $out/pytest.log
timeout -k 10 400 python -u bench_game.py --config game5pl --steps 5 --warmup 2 > $out/g.json 2> $out/g.log || { echo "bench failed"; tail -30 $out/g.log; exit 1; }
echo "game5pl: $(grep -o '"coordinate_ms[^}]*}' $out/g.json) $(grep -o 'sweeps (ms).*' $out/g.log) $(grep -o '"cold_first_sweep_ms[^,]*' $out/g.json)"
bash scripts/gpu_r4_window.sh game5pl r5q || exit 1
