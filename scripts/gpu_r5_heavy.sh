#!/bin/bash
# Round 5: heavy-tail preset (game5heavy: game5pl + entities of 45K x4 / 150K / 400K / 1M rows) -- solver routing
# (register-resident clusters), sweep times and the RE window. -> gpurun_out/r5heavy/
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5heavy
mkdir -p $out
timeout -k 10 600 python -u bench_game.py --config game5heavy --steps 3 --warmup 2 --log-level INFO > $out/g.json 2> $out/g.log || { echo "bench failed"; tail -30 $out/g.log; exit 1; }
grep -E "RE solver routing|sweeps \(ms\)|final training loss" $out/g.log | cut -c1-600
echo "game5heavy: $(grep -o '"coordinate_ms[^}]*}' $out/g.json) $(grep -o '"cold_first_sweep_ms[^,]*' $out/g.json)"
bash scripts/gpu_r4_window.sh game5heavy r5heavy > $out/window.log 2>&1 || { tail -20 $out/window.log; exit 1; }
grep -A14 "per-entity" $out/window.log | head -16
