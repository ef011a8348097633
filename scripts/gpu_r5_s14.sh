#!/bin/bash
# Round 5 step 14: btrsv reciprocal + readlane, back-map rows gathered from the solution: tests, game5pl windows.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5s14
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_game_gpu.py -k "trsv or row_space or materialize or game or rs_tron" -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
bash scripts/gpu_r4_window.sh game5pl r5s14 > $out/window.log 2>&1 || { tail -20 $out/window.log; exit 1; }
head -6 gpurun_out/r5s14_materialize_window.md
