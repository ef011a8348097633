#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python __graft_entry__.py build > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/pytest_kernels.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_kernels.log; exit 1; }
tail -1 gpurun_out/pytest_kernels.log
for cfg in "4 2" "4 4" "2 2"; do
  set -- $cfg
  PML_TL_WAVES=$1 PML_TL_WAVES_T=$2 timeout -k 10 300 python scripts/kbench.py --rows 16000000 --layout tiled --configs "0,0,0" > gpurun_out/kbp_$1_$2.log 2>&1 || { echo "kbench failed $cfg"; tail -30 gpurun_out/kbp_$1_$2.log; exit 1; }
  echo "waves fwd=$1 t=$2: $(tail -1 gpurun_out/kbp_$1_$2.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print("fwd %.3f t %.3f pass %.3f" % (r["fwd_ms"], r["t_ms"], r["pass_ms"]))')"
done
timeout -k 10 900 python bench.py > gpurun_out/bench_tiled.json 2> gpurun_out/bench_tiled.log || { echo "bench failed"; tail -40 gpurun_out/bench_tiled.log; exit 1; }
cat gpurun_out/bench_tiled.json
