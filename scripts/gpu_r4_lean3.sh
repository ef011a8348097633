#!/bin/bash
# rs_primal + GAME GPU tests, game5pl bench, torch-call attribution, then lean-kernel row-group A/B (micro).
set -o pipefail
mkdir -p gpurun_out/r4prim
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_game_gpu.py -x -q --timeout 200 --timeout-method thread -k "rs_primal or row_space or fused or lean or resident" > gpurun_out/r4prim/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r4prim/pytest.log; exit 1; }
tail -2 gpurun_out/r4prim/pytest.log
timeout -k 10 400 python -u bench_game.py --config game5pl --steps 5 --warmup 2 > gpurun_out/r4prim/g.json 2> gpurun_out/r4prim/g.log || { echo "bench failed"; tail -30 gpurun_out/r4prim/g.log; exit 1; }
cut -c130-330 gpurun_out/r4prim/g.json; grep "sweeps (ms)" gpurun_out/r4prim/g.log
timeout -k 10 400 python -u scripts/fe_torch_calls.py game5pl gpurun_out/fe_torch_calls.txt > gpurun_out/fe_torch_calls.log 2>&1 || { echo "torch calls failed"; tail -20 gpurun_out/fe_torch_calls.log; exit 1; }
timeout -k 10 300 python -u scripts/re_fused_bench.py 43000 lean > gpurun_out/r4prim/lean_base.log 2>&1 || { echo "micro failed"; tail -20 gpurun_out/r4prim/lean_base.log; exit 1; }
echo "base:"; grep -v amdgpu.ids gpurun_out/r4prim/lean_base.log | tail -1
for v in f2 h4 f2h4; do
  PML_RE_LIB=photon_ml_amd/ops/_lib/exp/libpml_re_$v.so timeout -k 10 300 python -u scripts/re_fused_bench.py 43000 lean > gpurun_out/r4prim/lean_$v.log 2>&1 || { echo "$v failed"; tail -20 gpurun_out/r4prim/lean_$v.log; exit 1; }
  echo "variant $v:"; grep -v amdgpu.ids gpurun_out/r4prim/lean_$v.log | tail -1
done
