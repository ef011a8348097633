#!/bin/bash
# Round 4: row-space classes up to 192 rows (rs_tron_big_kernel): GPU tests, then game5pl at PML_RS_NMAX 64/128/192.
set -o pipefail
mkdir -p gpurun_out/r4rsbig
export TMPDIR=/tmp
PML_CHECK_KERNEL_INPUTS=1 timeout -k 10 600 python -u -m pytest tests/test_game_gpu.py -x -q --timeout 300 --timeout-method thread -k "row_space or fused or resident" > gpurun_out/r4rsbig/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r4rsbig/pytest.log; exit 1; }
tail -1 gpurun_out/r4rsbig/pytest.log
for nm in 64 128 192; do
  PML_RS_NMAX=$nm timeout -k 10 300 python -u bench_game.py --config game5pl --steps 3 --warmup 2 > gpurun_out/r4rsbig/g5pl_$nm.json 2> gpurun_out/r4rsbig/g5pl_$nm.log || { echo "game5pl $nm failed"; tail -30 gpurun_out/r4rsbig/g5pl_$nm.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r4rsbig/g5pl_$nm.json')); print('nmax $nm', round(d['ms_per_step'],1), 'ms/sweep; min', round(d['sweep_ms_min'],1), d['coordinate_ms'], 'build', round(d['coordinate_build_s'],1), 's')"
done
