#!/bin/bash
# Pipelined Hessian-vector row pass of the lean RE kernel: microbenchmark A/B + model agreement.
set -o pipefail
out=gpurun_out/${1:-repipe}
mkdir -p $out
export TMPDIR=/tmp
RE_BENCH_ALL_ONLY=1 timeout -k 10 300 python -u scripts/re_fused_bench.py 43000 lean,leanp,lean,leanp > $out/micro.log 2>&1 || { echo "micro failed"; tail -20 $out/micro.log; exit 1; }
cat $out/micro.log
