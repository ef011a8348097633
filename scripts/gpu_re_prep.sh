#!/bin/bash
# Row-space prep before the fused launch: GAME GPU tests, game5pl bench, RE window timeline.
set -o pipefail
out=gpurun_out/${1:-reprep}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_game_gpu.py tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 400 python -u bench_game.py --config game5pl --steps 5 --warmup 2 > $out/g.json 2> $out/g.log || { echo "bench failed"; tail -30 $out/g.log; exit 1; }
cut -c1-330 $out/g.json; grep -o '"coordinate_ms[^}]*}' $out/g.json; grep "sweeps (ms)" $out/g.log
bash scripts/gpu_r4_window.sh game5pl ${1:-reprep} > $out/window.log 2>&1 || { echo "window failed"; tail -20 $out/window.log; exit 1; }
mv gpurun_out/${1:-reprep}_*_window.md $out/ 2>/dev/null; head -3 $out/${1:-reprep}_re_window.md
