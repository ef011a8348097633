#!/bin/bash
# TL sweep (fp64 LDS accumulators): block/tile bits and pipelining depth; then bench with the best default.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python __graft_entry__.py build > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
for cfg in "10 10 2" "10 10 4" "11 11 2" "11 10 2" "10 11 2" "11 11 4"; do
  set -- $cfg
  PML_TL_RBITS=$1 PML_TL_CBITS=$2 PML_TL_U=$3 timeout -k 10 300 python scripts/kbench.py --rows 16000000 --layout tiled --configs "0,0,0" > gpurun_out/kb64_$1_$2_$3.log 2>&1 || { echo "kbench failed $cfg"; tail -30 gpurun_out/kb64_$1_$2_$3.log; exit 1; }
  echo "rbits=$1 cbits=$2 U=$3: $(tail -1 gpurun_out/kb64_$1_$2_$3.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print("fwd %.3f t %.3f pass %.3f" % (r["fwd_ms"], r["t_ms"], r["pass_ms"]))')"
done
