#!/bin/bash
# TL kernels after the global-address-space / branchless fixes: parity tests + plain vs interleaved A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_kern.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_kern.log; exit 1; }
tail -1 gpurun_out/pytest_kern.log
timeout -k 10 500 python scripts/kbench.py --rows 16000000 --chunk-rows 1048576 --il 0 1 --tl-configs "2,4,0,1,0;4,4,0,1,0" > gpurun_out/kbench_il2.jsonl 2> gpurun_out/kbench_il2.log || { tail -30 gpurun_out/kbench_il2.log; exit 1; }
python3 - <<'PY'
import json
for line in open("gpurun_out/kbench_il2.jsonl"):
    r = json.loads(line)
    print("il=%d cfg=%s fwd %.3f t %.3f pass %.3f" % (r["il"], r["cfg"][1:3], r["fwd_ms"], r["t_ms"], r["pass_ms"]))
PY
