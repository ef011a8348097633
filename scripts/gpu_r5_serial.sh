#!/bin/bash
# Round 5: game5pl RE window with the row-space solve NOT overlapped (PML_RE_OVERLAP=0): each chain's own duration.
set -o pipefail
export TMPDIR=/tmp
PML_RE_OVERLAP=0 bash scripts/gpu_r4_window.sh game5pl r5serial > gpurun_out/r5serial_window.log 2>&1 || { tail -20 gpurun_out/r5serial_window.log; exit 1; }
head -14 gpurun_out/r5serial_re_window.md
grep -A60 "^| start ms" gpurun_out/r5serial_re_window.md | awk -F'|' '$3+0 > 0.3' | head -30
