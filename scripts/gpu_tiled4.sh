#!/bin/bash
# TL sweep: accumulator precision / block sizes / pipelining depth, then parity tests and bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python __graft_entry__.py build > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/pytest_kernels.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_kernels.log; exit 1; }
tail -1 gpurun_out/pytest_kernels.log
for cfg in "10 10 0 2" "10 10 1 2" "10 10 0 4" "11 11 0 2" "12 12 0 2" "12 12 0 4" "12 10 0 2" "10 12 0 2"; do
  set -- $cfg
  PML_TL_RBITS=$1 PML_TL_CBITS=$2 PML_TL_ACC64=$3 PML_TL_U=$4 timeout -k 10 300 python scripts/kbench.py --rows 16000000 --layout tiled --configs "0,0,0" > gpurun_out/kb_$1_$2_$3_$4.log 2>&1 || { echo "kbench failed $cfg"; tail -30 gpurun_out/kb_$1_$2_$3_$4.log; exit 1; }
  echo "rbits=$1 cbits=$2 acc64=$3 U=$4: $(tail -1 gpurun_out/kb_$1_$2_$3_$4.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print("fwd %.3f t %.3f pass %.3f" % (r["fwd_ms"], r["t_ms"], r["pass_ms"]))')"
done
