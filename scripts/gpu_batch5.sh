#!/bin/bash
# Row-sampled shard tests + the fused RE tests, the fused row-pass variants, game5pl per variant, and the
# down-sampled fixed-effect update (game5, rate 1.0 vs 0.1).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_downsample_gpu.py tests/test_sampling.py tests/test_game_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_b5.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_b5.log; exit 1; }
tail -2 gpurun_out/pytest_b5.log
for r in 1.0 0.1; do
  timeout -k 10 600 python -u bench_game.py --config game5 --steps 3 --warmup 2 --fe-down-sampling-rate $r > gpurun_out/game5_ds$r.json 2> gpurun_out/game5_ds$r.log || { echo "game5 ds $r failed"; tail -30 gpurun_out/game5_ds$r.log; exit 1; }
  echo "rate $r:"; cut -c1-160 gpurun_out/game5_ds$r.json; grep -o '"coordinate_ms".*' gpurun_out/game5_ds$r.json
done
timeout -k 10 300 python -u scripts/re_fused_bench.py 43000 2,3 > gpurun_out/re_fused_bench_v3.log 2>&1 || { echo "microbench failed"; tail -20 gpurun_out/re_fused_bench_v3.log; exit 1; }
cat gpurun_out/re_fused_bench_v3.log
PML_RE_ROWPASS=3 timeout -k 10 600 python -u -m pytest tests/test_game_gpu.py -x -q --timeout 300 --timeout-method thread -k "fused" > gpurun_out/pytest_v3.log 2>&1 || { echo "v3 pytest failed"; tail -40 gpurun_out/pytest_v3.log; exit 1; }
tail -1 gpurun_out/pytest_v3.log
for v in 3 2; do
  PML_RE_ROWPASS=$v timeout -k 10 600 python -u bench_game.py --config game5pl --steps 3 --warmup 2 > gpurun_out/game5pl_b4_v$v.json 2> gpurun_out/game5pl_b4_v$v.log || { echo "game5pl v$v failed"; tail -30 gpurun_out/game5pl_b4_v$v.log; exit 1; }
  echo "rowpass $v:"; cut -c1-200 gpurun_out/game5pl_b4_v$v.json
done
# upper bound of an LDS hot-column table in the forward: wide-round gathers of keys < H skipped (experiment build)
PML_GLM_LIB=photon_ml_amd/ops/_lib/libpml_glm_abl.so timeout -k 10 600 python -u scripts/kbench.py --rows 64000000 --reps 5 --tl-configs "2,4,3" --ablate 0 1056 2080 4128 8224 16416 > gpurun_out/kbench_hot_ablate_64M.jsonl 2> gpurun_out/kbench_hot_ablate_64M.log || { echo "kbench failed"; tail -20 gpurun_out/kbench_hot_ablate_64M.log; exit 1; }
cut -c1-260 gpurun_out/kbench_hot_ablate_64M.jsonl
