#!/bin/bash
# Round 6: kernel windows of the one-shot GAME run (build phases + cold first sweep), bf16 fixed effect.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6build
mkdir -p $out
export TMPDIR=/tmp
cd /tmp
PML_TRACE=1 PML_SYNC_TIMED=1 timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --stats -d $out/prof -o prof -- python3 $R/scripts/oneshot_profile.py --precisions bf16 > $out/run.md 2> $out/run.log || { echo "prof failed"; tail -30 $out/run.log; exit 1; }
cat $out/run.md | head -8
db=$(find $out/prof -name "*.db" | head -1)
export PML_WIN_TIMELINE=0
for w in "hottest-first relabel" "RE segmented: entity sort" "RE segmented: tiled layout" "FE global build: device layout" "RE per-entity: row-space batch" "RE per-entity: fused primal batch"; do
  f=$(echo "$w" | tr -c 'a-zA-Z0-9' '_')
  python3 $R/scripts/prof_window.py "$db" "$w" $out/win_$f.md > /dev/null && head -30 $out/win_$f.md
done
PML_WIN_INDEX=0 python3 $R/scripts/prof_window.py "$db" "Update coordinate global" $out/win_cold_fe.md > /dev/null && head -40 $out/win_cold_fe.md
PML_WIN_INDEX=0 python3 $R/scripts/prof_window.py "$db" "Update coordinate per-entity" $out/win_cold_re.md > /dev/null && head -40 $out/win_cold_re.md
PML_WIN_INDEX=1 python3 $R/scripts/prof_window.py "$db" "Update coordinate global" $out/win_warm_fe.md > /dev/null && head -12 $out/win_warm_fe.md
find $out/prof -name "*.csv" | head
rm -f $db
