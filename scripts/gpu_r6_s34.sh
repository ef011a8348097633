#!/bin/bash
# Round 6 step 34: device-complete phase times of the random-effect key build (PML_SYNC_TIMED=1), fresh process.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6s34
mkdir -p $out
export TMPDIR=/tmp
cd $R
PML_SYNC_TIMED=1 timeout -k 10 300 python -u scripts/oneshot_profile.py --precisions f64 --json $out/sync.json > $out/sync.md 2> $out/sync.log || { echo "oneshot failed"; tail -30 $out/sync.log; exit 1; }
grep -E "RE |build|upload|chunk" $out/sync.md | head -30
