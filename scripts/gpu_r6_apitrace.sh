#!/bin/bash
# Round 6: HIP runtime API time of the cold first sweep (where the first FE / RE updates' idle host time goes).
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6api
mkdir -p $out
export TMPDIR=/tmp
cd /tmp
PML_TRACE=1 timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --hip-runtime-trace -d $out/prof -o prof -- python3 $R/scripts/oneshot_profile.py --precisions bf16 > $out/run.md 2> $out/run.log || { echo "prof failed"; tail -30 $out/run.log; exit 1; }
head -5 $out/run.md
db=$(find $out/prof -name "*.db" | head -1)
python3 -c "
import sqlite3,sys; c=sqlite3.connect('$db')
print([r[0] for r in c.execute(\"select name from sqlite_master where type in ('view','table')\")])
for v in ('regions','kernels'):
    print(v, [r[1] for r in c.execute(f\"pragma table_info('{v}')\")])
print(list(c.execute('select * from regions limit 3')))
" > $out/schema.txt 2>&1
cat $out/schema.txt | cut -c1-600
for w in "Update coordinate global" "Update coordinate per-entity" "FE global build" "RE per-entity build"; do
  python3 $R/scripts/prof_api_window.py "$db" "$w" 0 > $out/api_$(echo "$w" | tr -c 'a-zA-Z0-9' '_').md && head -25 $out/api_$(echo "$w" | tr -c 'a-zA-Z0-9' '_').md
done
rm -f $db
