#!/bin/bash
# sqrt-sized transpose combine units: kernel tests, headline bench, kernel stats of the combine kernels.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_kernels_c.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_kernels_c.log; exit 1; }
tail -2 gpurun_out/pytest_kernels_c.log
timeout -k 10 900 python bench.py > gpurun_out/bench_combine.json 2> gpurun_out/bench_combine.log || { echo "bench failed"; tail -30 gpurun_out/bench_combine.log; exit 1; }
cat gpurun_out/bench_combine.json
cd /tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_comb -o prof --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 > $R/gpurun_out/prof_comb.log 2>&1 || { echo "prof failed"; tail -20 $R/gpurun_out/prof_comb.log; exit 1; }
f=$(find $R/gpurun_out/prof_comb -name "*kernel_stats.csv" | head -1)
head -8 "$f" | cut -c1-200
find $R/gpurun_out/prof_comb -name "*kernel_trace.csv" -delete
