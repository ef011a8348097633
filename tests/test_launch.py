"""Self-launch of the multi-GPU entry points: ``--gpus N`` without a launcher runs N ranks (never a mislabelled
1-rank record), and a launched world of the wrong size is an error."""
import json
import os
import subprocess
import sys

import pytest

from photon_ml_amd.parallel import launch

HERE = os.path.dirname(os.path.abspath(__file__))


def test_single_gpu_runs_in_process(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert launch.relaunch_if_needed(1, "bench.py", []) is None


def test_world_size_mismatch_is_an_error(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit) as e:
        launch.relaunch_if_needed(8, "bench.py", ["--gpus", "8"])
    assert e.value.code == 2
    assert launch.relaunch_if_needed(2, "bench.py", ["--gpus", "2"]) is None


def test_multi_gpu_without_launcher_starts_torchrun_child(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 7

    monkeypatch.setattr(launch.subprocess, "call", fake_call)
    assert launch.relaunch_if_needed(4, "bench.py", ["--gpus", "4", "--steps", "3"]) == 7
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_bench_game_two_ranks_on_one_device_refuse_or_say_rehearsal():
    """End to end on the CPU (gloo): 2 ranks share one physical device (the host CPU), so the record may not call
    them 2 GPUs — without --rehearsal the run refuses (exit 2); with it, n_gpus counts DEVICES (1) and n_ranks the
    ranks (2), and the record says rehearsal."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    base = [sys.executable, "bench_game.py", "--gpus", "2", "--config", "small", "--entities-per-gpu", "200",
            "--rows-per-entity", "4", "--re-dim", "10", "--re-nnz", "3", "--fe-dim", "500", "--fe-nnz", "5",
            "--steps", "1", "--warmup", "1", "--fe-iters", "2", "--re-iters", "2"]
    p = subprocess.run(base, cwd=os.path.dirname(HERE), env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode != 0, p.stderr[-2000:]     # the ranks exit 2; torchrun reports the failure
    assert "refusing to report them as 2 GPUs" in p.stderr
    p = subprocess.run(base + ["--rehearsal"], cwd=os.path.dirname(HERE), env=env, capture_output=True, text=True,
                       timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    rec = json.loads([ln for ln in p.stdout.splitlines() if ln.strip()][-1])
    assert rec["n_gpus"] == 1 and rec["n_ranks"] == 2 and rec["rehearsal"] is True
    assert rec["config"]["parallelism"] == "dp2+ep2"
    assert rec["config"]["global_batch"] == 2 * 200 * 4


def test_allreduce_algo_knob(monkeypatch):
    """--allreduce-algo / --tree-aggregate-depth -> NCCL_ALGO (the reference's treeAggregateDepth knob,
    GameEstimator.scala:111-114): depth >= 2 -> tree, 1 -> RCCL's choice; an explicit algorithm sticks; a user's
    own NCCL_ALGO wins."""
    from photon_ml_amd.parallel import dist
    monkeypatch.delenv("NCCL_ALGO", raising=False)
    monkeypatch.delenv("PML_NCCL_ALGO_SET", raising=False)
    monkeypatch.setattr(dist, "_EXPLICIT_ALGO", None)
    assert dist.set_allreduce_algo(tree_depth=2) == "tree" and os.environ["NCCL_ALGO"] == "Tree"
    assert dist.set_allreduce_algo(tree_depth=1) == "auto" and "NCCL_ALGO" not in os.environ
    assert dist.set_allreduce_algo("ring") == "ring" and os.environ["NCCL_ALGO"] == "Ring"
    assert dist.set_allreduce_algo(tree_depth=3) == "ring" and os.environ["NCCL_ALGO"] == "Ring"
    with pytest.raises(ValueError):
        dist.set_allreduce_algo("butterfly")
    monkeypatch.setattr(dist, "_EXPLICIT_ALGO", None)
    monkeypatch.delenv("PML_NCCL_ALGO_SET", raising=False)
    monkeypatch.setenv("NCCL_ALGO", "CollnetDirect")
    assert dist.set_allreduce_algo("tree") == "collnetdirect" and os.environ["NCCL_ALGO"] == "CollnetDirect"
    from photon_ml_amd.estimators.game_estimator import GameEstimator
    monkeypatch.delenv("NCCL_ALGO", raising=False)
    monkeypatch.setattr(dist, "_EXPLICIT_ALGO", None)
    GameEstimator(device="cpu").set_tree_aggregate_depth(2)
    assert os.environ.get("NCCL_ALGO") == "Tree"
    monkeypatch.delenv("NCCL_ALGO", raising=False)
