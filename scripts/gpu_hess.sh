#!/bin/bash
# Tall-narrow random effects: exact-Hessian MFMA kernel vs the sparse fused kernel on game5tall, the fused GPU
# tests, and one PMC pass with the MFMA counters on the production Hessian kernel.
set -o pipefail
mkdir -p gpurun_out/pmc_hess
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_game_gpu.py -x -q --timeout 300 --timeout-method thread -k "fused" > gpurun_out/pytest_hess.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_hess.log; exit 1; }
tail -1 gpurun_out/pytest_hess.log
for h in 1 0; do
  PML_RE_HESS=$h PML_SYNC_TIMING=1 timeout -k 10 600 python -u bench_game.py --config game5tall --steps 3 --warmup 2 --log-level DEBUG > gpurun_out/game5tall_h$h.json 2> gpurun_out/game5tall_h$h.log || { echo "game5tall h$h failed"; tail -30 gpurun_out/game5tall_h$h.log; exit 1; }
  echo "hess $h:"; grep -E "fused primal solve|row-space, " gpurun_out/game5tall_h$h.log | tail -2; cut -c1-200 gpurun_out/game5tall_h$h.json
done
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/pmc_hess -o p --output-format csv -- python3 bench_game.py --config game5tall --steps 1 --warmup 1 > gpurun_out/pmc_hess/run.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/pmc_hess/run.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc_hess "re_tron" gpurun_out/pmc_hess/summary.txt
find gpurun_out/pmc_hess -name "*.csv" -size +5M -delete
cat gpurun_out/pmc_hess/summary.txt
