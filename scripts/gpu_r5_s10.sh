#!/bin/bash
# Round 5 step 10: row-space class launches over 2 streams (PML_RS_STREAMS) vs 1 -- game5pl sweeps, RE window; RE tests.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5s10
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_game_gpu.py tests/test_fastpath_parity_gpu.py -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for ns in 1 2 1 2; do
  PML_RS_STREAMS=$ns timeout -k 10 400 python -u bench_game.py --config game5pl --steps 5 --warmup 2 > $out/g$ns.json 2> $out/g$ns.log || { echo "bench failed"; tail -30 $out/g$ns.log; exit 1; }
  echo "streams=$ns: $(grep -o '"coordinate_ms[^}]*}' $out/g$ns.json) $(grep -o 'sweeps (ms).*' $out/g$ns.log)"
done
bash scripts/gpu_r4_window.sh game5pl r5s10 > $out/window.log 2>&1 || { tail -20 $out/window.log; exit 1; }
head -12 gpurun_out/r5s10_re_window.md
