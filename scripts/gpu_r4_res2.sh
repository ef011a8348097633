#!/bin/bash
# Round 4: resident-kernel A/B (a: in-tree, b: no per-slot scheduling barrier, c: 8 slots) on the microbenchmark,
# then PMC passes of the in-tree resident vs streaming kernels (10K entities).
set -o pipefail
mkdir -p gpurun_out/r4res2
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/re_fused_bench.py 43000 stream,res > gpurun_out/r4res2/a.log 2>&1 || { echo "a failed"; tail -20 gpurun_out/r4res2/a.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4res2/a.log
PML_RE_LIB=photon_ml_amd/ops/_lib/exp/libpml_re_old.so timeout -k 10 300 python -u scripts/re_fused_bench.py 43000 stream > gpurun_out/r4res2/old.log 2>&1 || { echo "old failed"; tail -20 gpurun_out/r4res2/old.log; exit 1; }
echo "old streaming kernel (64-bit offsets):"; grep -v amdgpu.ids gpurun_out/r4res2/old.log | tail -1
for v in b c; do
  PML_RE_LIB=photon_ml_amd/ops/_lib/exp/libpml_re_$v.so timeout -k 10 300 python -u scripts/re_fused_bench.py 43000 res > gpurun_out/r4res2/$v.log 2>&1 || { echo "$v failed"; tail -20 gpurun_out/r4res2/$v.log; exit 1; }
  echo "variant $v:"; grep -v amdgpu.ids gpurun_out/r4res2/$v.log | tail -1
done
out=gpurun_out/r4res2/pmc
mkdir -p $out
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
            "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SCRATCH GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctrs -d $out/p$i -o p --output-format csv -- python3 scripts/re_fused_bench.py 10000 stream,res > $out/b$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $out/b$i.log; exit 1; }
done
python3 scripts/pmc_summary.py $out "re_tron" $out/summary.txt
find $out -name "*.csv" -size +20M -delete
cat $out/summary.txt
timeout -k 10 300 python -u scripts/fe_ops_profile.py game5pl gpurun_out/r4res2/fe_ops.txt > gpurun_out/r4res2/fe_ops.log 2>&1 || { echo "fe ops profile failed"; tail -20 gpurun_out/r4res2/fe_ops.log; }
