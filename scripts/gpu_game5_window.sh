#!/bin/bash
# Where does the GAME config-5 fixed-effect coordinate spend its wall time? kernel + marker trace, then the kernel
# busy fraction inside the last "coordinate global" region.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export PML_TRACE=1
cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --marker-trace -d /tmp/prof_g5w -o prof -- python3 $GRAFT_REPO_ROOT/bench_game.py --config game5 --steps 1 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_g5w.log 2>&1 || { echo "prof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof_g5w.log; exit 1; }
cd $GRAFT_REPO_ROOT && DB=$(find /tmp/prof_g5w -name "*.db" | head -1) && python scripts/prof_window.py $DB "Update coordinate global" gpurun_out/game5_fe_window.md && python scripts/prof_window.py $DB "Update coordinate per-entity" gpurun_out/game5_re_window.md
