#!/bin/bash
# RE coordinate critical path on game5pl: torch calls of one RE update + the RE window timeline (rocprofv3).
set -o pipefail
out=gpurun_out/${1:-recrit}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/fe_torch_calls.py game5pl $out/calls.txt > $out/calls.log 2>&1 || { echo "calls failed"; tail -20 $out/calls.log; exit 1; }
bash scripts/gpu_r4_window.sh game5pl ${1:-recrit} > $out/window.log 2>&1 || { echo "window failed"; tail -20 $out/window.log; exit 1; }
mv gpurun_out/${1:-recrit}_*_window.md $out/ 2>/dev/null; ls $out
