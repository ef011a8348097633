#!/bin/bash
# Round 6 step 32: the prefetched RE shard copy gated behind the FE upload -- GAME / RE / CLI / RCCL tests, the fresh-process
# one-shot (build + cold sweep) at both FE precisions, then game5pl warm sweeps.
set -o pipefail
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r6s32
mkdir -p $out
export TMPDIR=/tmp
cd $R
timeout -k 10 800 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_game_gpu.py tests/test_re_parity_gpu.py tests/test_fastpath_parity_gpu.py tests/test_cli_gpu.py tests/test_rccl_gpu.py tests/test_downsample_gpu.py > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 300 python -u scripts/oneshot_profile.py --precisions bf16,f64 --json $out/nosync.json > $out/nosync.md 2> $out/nosync.log || { echo "oneshot failed"; tail -30 $out/nosync.log; exit 1; }
grep -E "build|cold|warm-up|tiled layout" $out/nosync.md | head -30
for p in f64 bf16; do
  timeout -k 10 240 python3 bench_game.py --config game5pl --precision $p --steps 3 --warmup 2 > $out/g_$p.json 2> $out/g_$p.log || { echo "game $p failed"; tail -20 $out/g_$p.log; exit 1; }
  python3 - "$p" "$out/g_$p.json" <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print("game", sys.argv[1], "ms/sweep %.2f median %.2f" % (j["ms_per_step"], j["sweep_ms_median"]), {k: round(v, 2) for k, v in j["coordinate_ms"].items()}, "cold", round(j["cold_first_sweep_ms"], 1))
PY
done
