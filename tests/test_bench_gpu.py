"""The ``bench.py`` / ``bench_game.py`` driver contract at tiny sizes on the GPU: rank 0 prints ONE JSON line with
the fields the round driver reads (metric/config of BASELINE.json, whole-job value, timed steps, dtype)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _run(args, timeout=240):
    out = subprocess.run([sys.executable, *args], cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def test_bench_contract_tiny():
    rec = _run(["bench.py", "--steps", "2", "--warmup", "1", "--rows-per-gpu", "400000", "--features", "20000"])
    assert KEYS <= set(rec)
    assert rec["n_gpus"] == 1 and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["dtype"] == "bf16" and rec["higher_is_better"] is True and rec["scaling"] == "weak"
    assert rec["value"] > 0 and rec["ms_per_step"] > 0
    # value is the whole-job examples/s: rows x steps / elapsed
    assert abs(rec["value"] - rec["config"]["global_batch"] / (rec["ms_per_step"] / 1e3)) < 1e-6 * rec["value"]
    assert rec["config"]["parallelism"] == "dp1"


def test_bench_game_contract_tiny():
    rec = _run(["bench_game.py", "--steps", "1", "--warmup", "1", "--entities-per-gpu", "2000",
                "--rows-per-entity", "10", "--re-dim", "50", "--re-nnz", "5", "--fe-dim", "5000", "--fe-nnz", "10"])
    assert KEYS <= set(rec)
    assert rec["n_gpus"] == 1 and rec["value"] > 0 and rec["higher_is_better"] is True
