#!/bin/bash
# TL sweep: waves per WG x block/tile bits (fp64 LDS accumulation).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python __graft_entry__.py build > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/pytest_kernels.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_kernels.log; exit 1; }
tail -1 gpurun_out/pytest_kernels.log
PML_TL_WAVES=2 timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -k "tiled" > gpurun_out/pytest_kernels_w2.log 2>&1 || { echo "pytest w2 failed"; tail -40 gpurun_out/pytest_kernels_w2.log; exit 1; }
tail -1 gpurun_out/pytest_kernels_w2.log
for cfg in "4 10 10" "2 10 10" "2 11 11" "2 9 9" "4 9 9" "2 11 10" "2 10 11"; do
  set -- $cfg
  PML_TL_WAVES=$1 PML_TL_RBITS=$2 PML_TL_CBITS=$3 timeout -k 10 300 python scripts/kbench.py --rows 16000000 --layout tiled --configs "0,0,0" > gpurun_out/kbw_$1_$2_$3.log 2>&1 || { echo "kbench failed $cfg"; tail -30 gpurun_out/kbw_$1_$2_$3.log; exit 1; }
  echo "waves=$1 rbits=$2 cbits=$3: $(tail -1 gpurun_out/kbw_$1_$2_$3.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print("fwd %.3f t %.3f pass %.3f" % (r["fwd_ms"], r["t_ms"], r["pass_ms"]))')"
done
