#!/bin/bash
# Timed-window kernel profile of the headline bench: kernel + marker trace, then kernel busy time inside the
# "bench timed steps" roctx region (excludes data generation and the one-time tiled-layout build).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export PML_TRACE=1
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace -d /tmp/prof_bw -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --rows-per-gpu 32000000 --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_bw.log 2>&1 || { echo "prof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof_bw.log; exit 1; }
cd $GRAFT_REPO_ROOT && DB=$(find /tmp/prof_bw -name "*.db" | head -1) && python scripts/prof_window.py $DB "bench timed steps" gpurun_out/bench_32M_timed_window.md && cat gpurun_out/bench_32M_timed_window.md
