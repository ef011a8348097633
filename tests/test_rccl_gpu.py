"""RCCL on one MI355X: the multi-rank code paths (bucketed async gradient all-reduce overlapped with the transpose
kernels, TRON Hessian-vector reductions, feature-sharded all-gather / reduce-scatter, entity-sharded GAME routing
with device all-to-all) executed through real ``nccl`` (= RCCL) collectives with a one-rank group
(``PML_FORCE_DIST=1``), compared with the same computation without a process group.

A one-rank sum is the identity, so the data-parallel GLM iterates must be BITWISE equal (the bucketed path
reduces tile-independent slices: same bits as the one-shot path); the entity-sharded GAME path reorders rows
through the router, so it is compared to 1e-9.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(mode, out, env_extra):
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_port()), **env_extra)
    p = subprocess.run([sys.executable, "-u", os.path.join(HERE, "nccl_worker.py"), mode, str(out)], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert f"{mode} ok" in p.stdout


def test_rccl_single_rank_paths_match_local(tmp_path):
    _run("forced", tmp_path, {"PML_FORCE_DIST": "1", "PML_DIST_BACKEND": "nccl"})
    _run("plain", tmp_path, {"PML_FORCE_DIST": "0"})
    for name in ("lbfgs", "tron"):
        a, b = np.load(tmp_path / f"forced_{name}_w.npy"), np.load(tmp_path / f"plain_{name}_w.npy")
        assert np.array_equal(a, b), (name, np.abs(a - b).max())
        assert np.array_equal(np.load(tmp_path / f"forced_{name}_f.npy"), np.load(tmp_path / f"plain_{name}_f.npy"))
    # feature-sharded state: the same margin-space line search as the replicated path (trials from the cached
    # margins, z0 + t zd in fp64); only the two-loop's inner products are summed in another order (sharded Gram)
    a, b = np.load(tmp_path / "forced_fsdp_w.npy"), np.load(tmp_path / "plain_fsdp_w.npy")
    assert np.abs(a - b).max() <= 1e-10 * np.abs(b).max(), np.abs(a - b).max()
    for part in ("game_fe", "game_eval", "game_per-user", "game_per-item"):
        a, b = np.load(tmp_path / f"forced_{part}.npy"), np.load(tmp_path / f"plain_{part}.npy")
        np.testing.assert_allclose(a, b, rtol=1e-8, atol=1e-9, err_msg=part)


def test_bench_through_torchrun_rccl_one_rank():
    """bench.py exactly as the driver launches it for N > 1 (torchrun, RCCL), with a one-rank group."""
    import json
    env = dict(os.environ, PML_FORCE_DIST="1")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "1",
                        "--steps", "2", "--warmup", "1", "--rows-per-gpu", "400000", "--features", "20000"],
                       cwd=os.path.dirname(HERE), env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-4000:]
    assert "overlapped" in p.stderr, p.stderr[-2000:]
    rec = json.loads([ln for ln in p.stdout.splitlines() if ln.strip()][-1])
    assert rec["n_gpus"] == 1 and rec["evals_per_step"] == 1.0 and rec["value"] > 0
