#!/bin/bash
# Round 4: one-wave-per-entity tall-narrow TRON (re_tron_tall_kernel): fused GPU tests + game5tall RE window.
set -o pipefail
mkdir -p gpurun_out/r4tall
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_game_gpu.py -x -q --timeout 120 --timeout-method thread -k "fused" > gpurun_out/r4tall/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r4tall/pytest.log; exit 1; }
tail -1 gpurun_out/r4tall/pytest.log
bash scripts/gpu_r4_window.sh game5tall ${1:-game5tall_r4}
grep -E "RE stats" gpurun_out/prof_${1:-game5tall_r4}.log | cut -c1-300
