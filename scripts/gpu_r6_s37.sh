#!/bin/bash
# Round 6 step 37: final-tree kernel statistics (rocprofv3 --kernel-trace --stats): the headline bench and game5pl fp64.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6s37
mkdir -p $out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/head -o head --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --game off --configs-extra off > $out/head.json 2> $out/head.log || { echo "headline prof failed"; tail -20 $out/head.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/g64 -o g64 --output-format csv -- python3 $R/bench_game.py --config game5pl --precision f64 --steps 3 --warmup 2 > $out/g64.json 2> $out/g64.log || { echo "game prof failed"; tail -20 $out/g64.log; exit 1; }
for d in head g64; do
  f=$(find $out/$d -name "*kernel_stats.csv" | head -1)
  cp "$f" $out/${d}_kernel_stats.csv
  python3 - "$out/${d}_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(sys.argv[1].split("/")[-1], "kernels:", len(rows), "total ms: %.1f" % (tot / 1e6))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print("  %9.2f ms %6s calls %5.1f %%  %s" % (float(r["TotalDurationNs"]) / 1e6, r["Calls"], 100 * float(r["TotalDurationNs"]) / tot, r["Name"][:90]))
PY
done
find $out -name "*.csv" ! -name "*_kernel_stats.csv" -delete
