#!/bin/bash
# Round 5 final: GPU test tier, smoke(), bench.py (driver contract, 1 GPU), game5pl / game5heavy windows.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5final
mkdir -p $out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $out/pytest.log | tail -20; tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 900 python -u bench.py > $out/bench.json 2> $out/bench.log || { echo "bench failed"; tail -30 $out/bench.log; exit 1; }
grep '^{' $out/bench.json | cut -c1-900
bash scripts/gpu_r4_window.sh game5pl r5final > $out/window.log 2>&1 || { tail -20 $out/window.log; exit 1; }
head -3 gpurun_out/r5final_re_window.md
