#!/bin/bash
# Device-order gradient scratch, dense-bucket fused TRON, feature-sharded margin line search: tests, the headline
# bench, feature-sharded vs replicated (16M rows), and the game5 fixed-effect window (kernels + idle gaps).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_downsample_gpu.py tests/test_rccl_gpu.py tests/test_game_gpu.py -x -q --timeout 300 --timeout-method thread -k "not test_fused_entity_tron_matches_pass_path" > gpurun_out/pytest_b6.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_b6.log; exit 1; }
tail -2 gpurun_out/pytest_b6.log
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --game off > gpurun_out/bench_b6.json 2> gpurun_out/bench_b6.log || { echo "bench failed"; tail -20 gpurun_out/bench_b6.log; exit 1; }
cut -c1-300 gpurun_out/bench_b6.json
for st in feature-sharded replicated; do
  timeout -k 10 300 python -u bench.py --rows-per-gpu 16000000 --steps 5 --warmup 2 --game off --optimizer-state $st > gpurun_out/bench_16M_$st.json 2> gpurun_out/bench_16M_$st.log || { echo "bench $st failed"; tail -20 gpurun_out/bench_16M_$st.log; exit 1; }
  cut -c1-300 gpurun_out/bench_16M_$st.json
done
for r in 1.0 0.1; do
  timeout -k 10 600 python -u bench_game.py --config game5 --steps 3 --warmup 2 --fe-down-sampling-rate $r > gpurun_out/game5_ds$r.json 2> gpurun_out/game5_ds$r.log || { echo "game5 ds $r failed"; tail -30 gpurun_out/game5_ds$r.log; exit 1; }
  echo "rate $r:"; cut -c1-200 gpurun_out/game5_ds$r.json; grep -o '"coordinate_ms".*' gpurun_out/game5_ds$r.json
done
PML_GLM_LIB=photon_ml_amd/ops/_lib/libpml_glm_abl.so timeout -k 10 600 python -u scripts/kbench.py --rows 64000000 --reps 5 --tl-configs "2,4,3" --ablate 0 4160 8256 16448 32832 > gpurun_out/kbench_hot_uniform_64M.jsonl 2> gpurun_out/kbench_hot_uniform_64M.log || { echo "kbench failed"; tail -20 gpurun_out/kbench_hot_uniform_64M.log; exit 1; }
cut -c1-100 gpurun_out/kbench_hot_uniform_64M.jsonl
cd /tmp
PML_TRACE=1 timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace -d $R/gpurun_out/prof_g5 -o prof -- python3 $R/bench_game.py --config game5 --steps 1 --warmup 2 > $R/gpurun_out/gaps_g5.json 2> $R/gpurun_out/gaps_g5.log || { echo "game prof failed"; tail -30 $R/gpurun_out/gaps_g5.log; exit 1; }
db=$(find $R/gpurun_out/prof_g5 -name "*.db" | head -1)
python3 $R/scripts/prof_window.py "$db" "Update coordinate global" $R/gpurun_out/game5_fe_window_b6.md > /dev/null && head -32 $R/gpurun_out/game5_fe_window_b6.md
rm -rf $R/gpurun_out/prof_g5
