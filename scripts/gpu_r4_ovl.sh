#!/bin/bash
# Row-space solve overlapped with the fused solve (side stream), rs_tron margins fused, masked to_primal:
# GAME + row-space kernel GPU tests, game5pl A/B (PML_RE_OVERLAP=0 / 1), RE window.
set -o pipefail
mkdir -p gpurun_out/r4ovl
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_game_gpu.py tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -k "game or rs_tron or row_space or fused or lean or batched" > gpurun_out/r4ovl/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r4ovl/pytest.log; exit 1; }
tail -2 gpurun_out/r4ovl/pytest.log
for ov in 0 1; do
  PML_RE_OVERLAP=$ov timeout -k 10 400 python -u bench_game.py --config game5pl --steps 5 --warmup 2 > gpurun_out/r4ovl/g$ov.json 2> gpurun_out/r4ovl/g$ov.log || { echo "game5pl $ov failed"; tail -30 gpurun_out/r4ovl/g$ov.log; exit 1; }
  echo "overlap $ov: $(cut -c1-330 gpurun_out/r4ovl/g$ov.json)"
  grep "sweeps (ms)" gpurun_out/r4ovl/g$ov.log
done
bash scripts/gpu_r4_window.sh game5pl g5pl_ovl
