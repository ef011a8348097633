#!/bin/bash
# game5pl phase timings (DEBUG, synchronized phases) under a kernel trace, then rs_tron PMC passes.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
PML_SYNC_TIMING=1 timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_g5pl -o prof -- python3 $R/bench_game.py --config game5pl --steps 1 --warmup 2 --log-level DEBUG > $R/gpurun_out/prof_g5pl.json 2> $R/gpurun_out/prof_g5pl.log || { echo "prof failed"; tail -30 $R/gpurun_out/prof_g5pl.log; exit 1; }
cat $R/gpurun_out/prof_g5pl.json
grep -E "row-space|primal|iteration|RE stats" $R/gpurun_out/prof_g5pl.log | cut -c1-300 | tail -30
f=$(find $R/gpurun_out/prof_g5pl -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:10.2f} ms {int(r["Calls"]):8d} {r["Name"][:150]}')
PY
cd $R && bash scripts/gpu_pmc_rs.sh
