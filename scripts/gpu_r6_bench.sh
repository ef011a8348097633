#!/bin/bash
# Round 6: driver-contract bench (headline + GAME + configs 3/4), smoke.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6bench
mkdir -p $out
timeout -k 10 200 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_kernels_gpu.py -k "warmup" > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 900 python -u bench.py > $out/bench.json 2> $out/bench.log || { echo "bench failed"; tail -40 $out/bench.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$out/bench.json') if l.startswith('{')][-1])
for k,v in d.items():
    if k not in ('config',): print(k, json.dumps(v)[:300])
"
grep -E "ms/step|failed|error" $out/bench.log | head -20
