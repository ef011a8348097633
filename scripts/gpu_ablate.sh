#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 400 python scripts/kbench.py --rows 8000000 --chunk-rows 1048576 --ablate 0 1 2 3 > gpurun_out/ablate.jsonl 2> gpurun_out/ablate.log || { tail -30 gpurun_out/ablate.log; exit 1; }
cat gpurun_out/ablate.jsonl
rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE -d gpurun_out/pmc -o pmc --output-format csv -- python3 scripts/kbench.py --rows 4000000 --reps 1 > gpurun_out/pmc/kb.json 2> gpurun_out/pmc/kb.log || { echo "pmc run failed"; tail -20 gpurun_out/pmc/kb.log; }
ls gpurun_out/pmc
