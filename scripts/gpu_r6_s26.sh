#!/bin/bash
# Round 6 step 26: row-space margins written straight into the RE update's score vector, fp64 zero point read in
# place -- GAME / RE / fast-path tests, then game5pl at both FE precisions (two runs each).
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6s26
mkdir -p $out
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_game_gpu.py tests/test_re_parity_gpu.py tests/test_fastpath_parity_gpu.py tests/test_lbfgs_plan_gpu.py > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2; do
  for p in f64 bf16; do
    timeout -k 10 240 python3 bench_game.py --config game5pl --precision $p --steps 5 --warmup 2 > $out/g_$p.$rep.json 2> $out/g_$p.$rep.log || { echo "game $p failed"; tail -20 $out/g_$p.$rep.log; exit 1; }
    python3 - "$p" "$out/g_$p.$rep.json" <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print("game", sys.argv[1], "ms/sweep %.2f median %.2f" % (j["ms_per_step"], j["sweep_ms_median"]), {k: round(v, 2) for k, v in j["coordinate_ms"].items()})
PY
  done
done
