#!/bin/bash
# Round 6 final tree: whole GPU test tier + smoke.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6s39
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $out/pytest.log | tail -20; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
