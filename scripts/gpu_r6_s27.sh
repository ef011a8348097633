#!/bin/bash
# Round 6 step 27: btrsv staging with 8 loads in flight -- its tests, then the fp64 game5pl windows (materialise, RE timeline).
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6s27
mkdir -p $out
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "trsv or primal or rs_" tests/test_re_parity_gpu.py > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
cd /tmp
PML_TRACE=1 timeout -k 10 500 rocprofv3 --kernel-trace --marker-trace -d $out/prof -o prof -- python3 $R/bench_game.py --config game5pl --precision f64 --steps 3 --warmup 2 > $out/run.json 2> $out/run.log || { echo "prof failed"; tail -30 $out/run.log; exit 1; }
grep -E "sweeps \(ms\)" $out/run.log | tail -2
db=$(find $out/prof -name "*.db" | head -1)
python3 $R/scripts/prof_window.py "$db" "materialize model" $out/win_mat.md > /dev/null; sed -n 1,12p $out/win_mat.md
python3 $R/scripts/prof_window.py "$db" "Update coordinate per-entity" $out/win_re.md > /dev/null; sed -n 1,8p $out/win_re.md
python3 $R/scripts/prof_window.py "$db" "timed sweeps" $out/win_sweeps.md > /dev/null; sed -n 1,2p $out/win_sweeps.md
rm -f $db
