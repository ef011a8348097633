#!/bin/bash
# Round 5 step 3: row-space / lean split A/B on game5pl, then the RE / FE / materialisation windows.
set -o pipefail
export TMPDIR=/tmp
bash scripts/gpu_r5_rsmix.sh || exit 1
bash scripts/gpu_r4_window.sh game5pl r5a || exit 1
