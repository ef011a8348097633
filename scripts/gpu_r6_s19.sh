#!/bin/bash
# Round 6 step 19: game5pl at fp64 FE storage -- where the timed window's time goes (sweeps, materialisation, FE, RE).
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6s19
mkdir -p $out
export TMPDIR=/tmp
cd /tmp
PML_TRACE=1 timeout -k 10 500 rocprofv3 --kernel-trace --marker-trace -d $out/prof -o prof -- python3 $R/bench_game.py --config game5pl --precision f64 --steps 3 --warmup 2 > $out/run.json 2> $out/run.log || { echo "prof failed"; tail -30 $out/run.log; exit 1; }
grep -E "sweeps \(ms\)|coordinate" $out/run.log | tail -12
db=$(find $out/prof -name "*.db" | head -1)
export PML_WIN_TIMELINE=0
python3 $R/scripts/prof_window.py "$db" "materialize model" $out/win_mat.md > /dev/null; sed -n 1,40p $out/win_mat.md
PML_WIN_TIMELINE=1 python3 $R/scripts/prof_window.py "$db" "materialize model" $out/win_mat_tl.md > /dev/null
python3 $R/scripts/prof_window.py "$db" "timed sweeps" $out/win_sweeps.md > /dev/null; sed -n 1,60p $out/win_sweeps.md
python3 $R/scripts/prof_window.py "$db" "Update coordinate global" $out/win_fe.md > /dev/null; sed -n 1,30p $out/win_fe.md
python3 $R/scripts/prof_window.py "$db" "Update coordinate per-entity" $out/win_re.md > /dev/null; sed -n 1,30p $out/win_re.md
rm -f $db
