#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_game_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_b4.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_b4.log; exit 1; }
tail -2 gpurun_out/pytest_b4.log
timeout -k 10 300 python -u scripts/re_fused_bench.py 43000 2,3 > gpurun_out/re_fused_bench_v3.log 2>&1 || { echo "microbench failed"; tail -20 gpurun_out/re_fused_bench_v3.log; exit 1; }
cat gpurun_out/re_fused_bench_v3.log
PML_RE_ROWPASS=3 timeout -k 10 600 python -u -m pytest tests/test_game_gpu.py -x -q --timeout 300 --timeout-method thread -k "fused" > gpurun_out/pytest_v3.log 2>&1 || { echo "v3 pytest failed"; tail -40 gpurun_out/pytest_v3.log; exit 1; }
tail -1 gpurun_out/pytest_v3.log
for v in 3 2; do
  PML_RE_ROWPASS=$v timeout -k 10 600 python -u bench_game.py --config game5pl --steps 3 --warmup 2 > gpurun_out/game5pl_b4_v$v.json 2> gpurun_out/game5pl_b4_v$v.log || { echo "game5pl v$v failed"; tail -30 gpurun_out/game5pl_b4_v$v.log; exit 1; }
  echo "rowpass $v:"; cut -c1-200 gpurun_out/game5pl_b4_v$v.json
done
bash scripts/gpu_cfg34.sh r3
