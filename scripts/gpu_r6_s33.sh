#!/bin/bash
# Round 6 final tree (lazy RE layout + gated prefetch): whole GPU test tier, smoke, the driver-contract bench, then a 2-rank rehearsal (gloo, both
# ranks on cuda:0) of the entity-sharded GAME path and the DP headline.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6s33
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $out/pytest.log | tail -20; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.log || { echo "bench failed"; tail -30 $out/bench.log; exit 1; }
python3 - $out/bench.json <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
keys = ["value", "ms_per_step", "game5pl_ms_per_sweep", "game5pl_sweep_ms_median", "game5pl_coordinate_ms",
        "game5pl_f64_ms_per_sweep", "game5pl_f64_sweep_ms_median", "game5pl_f64_coordinate_ms",
        "game5pl_cold_first_sweep_ms", "game5pl_f64_cold_first_sweep_ms", "game5pl_coordinate_build_s",
        "game5pl_f64_coordinate_build_s", "game5pl_one_shot_s", "game5pl_f64_one_shot_s", "owlqn10m_f64_ms_per_step",
        "owlqn10m_bf16_ms_per_step", "tron_poisson_f64_ms_per_step", "tron_poisson_bf16_ms_per_step"]
for k in keys:
    print(k, j.get(k))
PY
PML_DIST_BACKEND=gloo timeout -k 10 600 python -u bench_game.py --gpus 2 --rehearsal --config game5pl --entities-per-gpu 500000 --steps 2 --warmup 1 --log-level INFO > $out/placed.json 2> $out/placed.log || { echo "game rehearsal failed"; tail -40 $out/placed.log; exit 1; }
grep -E "rows placed|coordinates built|sweeps \(ms\)" $out/placed.log | cut -c1-300
PML_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --rehearsal --rows-per-gpu 8000000 --steps 3 --warmup 2 --game off > $out/headline.json 2> $out/headline.log || { echo "headline rehearsal failed"; tail -30 $out/headline.log; exit 1; }
tail -c 600 $out/headline.json
