#!/bin/bash
# MFMA evidence: timing + parity of gemm_nt / batched Gram, then one PMC pass with the MFMA counters.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_mfma
export TMPDIR=/tmp
timeout -k 10 300 python3 $R/scripts/mfma_bench.py > $R/gpurun_out/mfma_bench.log 2>&1 || { echo "mfma bench failed"; tail -20 $R/gpurun_out/mfma_bench.log; exit 1; }
grep -v amdgpu.ids $R/gpurun_out/mfma_bench.log
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_mfma -o p --output-format csv -- python3 $R/scripts/mfma_bench.py > $R/gpurun_out/pmc_mfma/run.log 2>&1 || { echo "pmc failed"; tail -20 $R/gpurun_out/pmc_mfma/run.log; exit 1; }
cd $R && python3 scripts/pmc_summary.py gpurun_out/pmc_mfma "mfma|spmm" gpurun_out/pmc_mfma/summary.txt
find gpurun_out/pmc_mfma -name "*.csv" -size +5M -delete
