#!/bin/bash
# Round 6: phase table of the one-shot GAME run (coordinate build + cold first sweep), fresh process.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6oneshot
mkdir -p $out
PML_SYNC_TIMED=1 timeout -k 10 300 python -u scripts/oneshot_profile.py --precisions bf16,f64 --json $out/phases.json --cprofile $out/cprofile.txt > $out/phases.md 2> $out/phases.log || { echo "oneshot failed"; tail -30 $out/phases.log; exit 1; }
cat $out/phases.md
timeout -k 10 300 python -u scripts/oneshot_profile.py --precisions bf16,f64 --json $out/nosync.json > $out/nosync.md 2> $out/nosync.log || { echo "oneshot nosync failed"; tail -30 $out/nosync.log; exit 1; }
grep -E "coordinate build" $out/nosync.md
