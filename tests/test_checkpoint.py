"""Checkpoint / resume of GAME coordinate descent (new — the reference has no mid-training
checkpoints): an interrupted fit resumed from the last coordinate update equals an uninterrupted one."""
from collections import OrderedDict

import numpy as np
import pytest
import torch

from photon_ml_amd.algorithm.coordinate_descent import CoordinateDescent
from photon_ml_amd.algorithm.coordinates import FixedEffectCoordinate, RandomEffectCoordinate
from photon_ml_amd.data.game_data import generate_game_data
from photon_ml_amd.data.random_effect import FixedEffectDataConfiguration, RandomEffectDataConfiguration
from photon_ml_amd.evaluation.evaluators import build_evaluator
from photon_ml_amd.optimization.config import GLMOptimizationConfiguration, OptimizerConfig, RegularizationContext
from photon_ml_amd.utils.checkpoint import Checkpointer


class Interrupt(Exception):
    pass


def _setup(seed=5):
    data, _ = generate_game_data(n_rows=1500, n_users=20, seed=seed, task="LOGISTIC_REGRESSION")
    val, _ = generate_game_data(n_rows=600, n_users=20, seed=seed + 1, task="LOGISTIC_REGRESSION")
    cfg = GLMOptimizationConfiguration(OptimizerConfig("TRON", 30, 1e-9), RegularizationContext("L2"), 1.0)
    coords = OrderedDict([
        ("g", FixedEffectCoordinate("g", data, FixedEffectDataConfiguration("global"), cfg, "LOGISTIC_REGRESSION",
                                    device="cpu")),
        ("u", RandomEffectCoordinate("u", data, RandomEffectDataConfiguration("userId", "user"), cfg,
                                     "LOGISTIC_REGRESSION", device="cpu")),
        ("i", RandomEffectCoordinate("i", data, RandomEffectDataConfiguration("itemId", "item"), cfg,
                                     "LOGISTIC_REGRESSION", device="cpu")),
    ])
    evs = [build_evaluator("AUC", val.response, val.offsets, val.weights)]
    return data, val, coords, evs


def test_resume_equals_uninterrupted(tmp_path):
    data, val, coords, evs = _setup()
    full_model, full_evals = CoordinateDescent(coords, None, val, evs).run(3)

    data, val, coords, evs = _setup()
    calls = {"n": 0}

    def bomb(rec):
        calls["n"] += 1
        if calls["n"] == 5:  # die in the middle of the second sweep
            raise Interrupt()
    ck = Checkpointer(str(tmp_path), "cd")
    with pytest.raises(Interrupt):
        CoordinateDescent(coords, None, val, evs, event_callback=bomb).run(3, checkpointer=ck, tag="t")
    st = ck.load_cd()
    assert (st["iteration"], st["next"]) == (1, 1)  # saved after "g" of sweep 2; "u" was interrupted

    data, val, coords, evs = _setup()
    model, evals = CoordinateDescent(coords, None, val, evs).run(3, checkpointer=Checkpointer(str(tmp_path), "cd"),
                                                                tag="t")
    assert abs(evals[0][1] - full_evals[0][1]) < 1e-9
    wa = model.get("g").glm.coefficients.means
    wb = full_model.get("g").glm.coefficients.means
    assert torch.allclose(wa, wb, atol=1e-8)
    a, b = model.get("u"), full_model.get("u")
    assert np.array_equal(a.keys, b.keys) and np.allclose(a.values, b.values, atol=1e-8)


def test_tag_mismatch_starts_fresh(tmp_path):
    data, val, coords, evs = _setup()
    ck = Checkpointer(str(tmp_path), "cd")
    CoordinateDescent(coords, None, val, evs).run(1, checkpointer=ck, tag="a")
    st = ck.load_cd()
    assert st["iteration"] == 1 and st["tag"] == "a"
    cd = CoordinateDescent(coords, None, val, evs)
    cd.run(1, checkpointer=ck, tag="b")
    assert len(cd.history) == 3  # all three coordinates re-run


@pytest.mark.parametrize("opt_name", ["LBFGS", "OWLQN", "TRON"])
def test_optimizer_resume_is_bitwise(tmp_path, opt_name):
    """Mid-solve optimizer checkpoint (coefficients, L-BFGS history, TRON radius, tolerances) -> a fresh optimizer
    resumed from disk produces exactly the iterates of the uninterrupted run."""
    import torch
    from photon_ml_amd.data.synthetic import generate_glm_data
    from photon_ml_amd.function.losses import LOGISTIC
    from photon_ml_amd.function.objective import GLMObjective
    from photon_ml_amd.ops.reference import TorchGLMData
    from photon_ml_amd.optimization.lbfgs import LBFGS, OWLQN
    from photon_ml_amd.optimization.tron import TRON
    from photon_ml_amd.utils.checkpoint import Checkpointer
    data, _ = generate_glm_data("LOGISTIC_REGRESSION", 1500, 30, density=0.3, seed=5)
    gd = TorchGLMData(data, "cpu")
    obj = GLMObjective(LOGISTIC, l2_weight=0.0 if opt_name == "OWLQN" else 1.0)
    make = {"LBFGS": lambda: LBFGS(tolerance=0.0, max_iterations=50),
            "OWLQN": lambda: OWLQN(2.0, tolerance=0.0, max_iterations=50),
            "TRON": lambda: TRON(tolerance=0.0, max_iterations=50)}[opt_name]
    w0 = torch.zeros(30, dtype=torch.float64)
    a = make()
    a.start(obj, gd, w0)
    ref = [a.step(obj, gd).coefficients.clone() for _ in range(8)]
    b = make()
    b.start(obj, gd, w0)
    for _ in range(4):
        b.step(obj, gd)
    ck = Checkpointer(str(tmp_path), "opt")
    ck.save_optimizer(b)
    c = make()
    assert ck.load_optimizer(c)
    got = [c.step(obj, gd).coefficients.clone() for _ in range(4)]
    for x, y in zip(ref[4:], got):
        assert torch.equal(x, y)


def test_glm_problem_checkpointed_run_resumes(tmp_path):
    """GLMOptimizationProblem with checkpointing: a run killed after k iterations and restarted from the saved
    optimizer state ends at the same model as an uninterrupted run."""
    from photon_ml_amd.data.synthetic import generate_glm_data
    from photon_ml_amd.ops.reference import TorchGLMData
    from photon_ml_amd.optimization.config import (GLMOptimizationConfiguration, OptimizerConfig,
                                                   RegularizationContext)
    from photon_ml_amd.optimization.problem import GLMOptimizationProblem
    from photon_ml_amd.utils.checkpoint import Checkpointer
    data, _ = generate_glm_data("LOGISTIC_REGRESSION", 1500, 30, density=0.3, seed=9)
    gd = TorchGLMData(data, "cpu")
    cfg = GLMOptimizationConfiguration(OptimizerConfig("LBFGS", 30, 1e-12), RegularizationContext("L2"), 1.0)
    full = GLMOptimizationProblem(cfg, "LOGISTIC_REGRESSION").run(gd)
    # "crashed" run: only 7 iterations, checkpointing every 2 (last save at iteration 6)
    short = GLMOptimizationConfiguration(OptimizerConfig("LBFGS", 7, 1e-12), RegularizationContext("L2"), 1.0)
    ck = Checkpointer(str(tmp_path), "glm")
    GLMOptimizationProblem(short, "LOGISTIC_REGRESSION").enable_checkpointing(ck, 2).run(gd)
    resumed = GLMOptimizationProblem(cfg, "LOGISTIC_REGRESSION").enable_checkpointing(ck, 2).run(gd)
    assert torch.equal(full.coefficients.means, resumed.coefficients.means)


def test_entity_ids_round_trip_any_characters_and_world_size_guard(tmp_path, monkeypatch):
    from photon_ml_amd.utils import checkpoint as ck
    ids = ["a", "", "line\nbreak", "ünïcode", "x" * 300]
    arr = ck._strings_to_array(ids)
    assert list(ck._array_to_strings(arr, len(ids))) == ids
    with pytest.raises(ValueError):
        ck._array_to_strings(arr, len(ids) - 1)
    c = ck.Checkpointer(str(tmp_path))
    c.save({"x": np.zeros(1)}, {"model": {"coordinates": []}, "iteration": 0, "next": 0, "world_size": 2})
    with pytest.raises(RuntimeError, match="world size"):
        c.load_cd()


def test_first_format_checkpoint_still_loads(tmp_path):
    """A version-less checkpoint of the first format (entity ids joined by newlines, no world size) resumes."""
    from photon_ml_amd.utils import checkpoint as ck
    ids = ["u1", "u2", "u3"]
    legacy = np.frombuffer("\n".join(ids).encode("utf-8"), dtype=np.uint8).copy()
    meta = {"model": {"coordinates": [{"id": "per-user", "kind": "random", "shard": "s", "re_type": "userId",
                                       "task": "LINEAR_REGRESSION", "dim": 4, "n_entities": 3}]},
            "iteration": 1, "next": 0}
    arrays = {"model/per-user.keys": np.array([0, 5, 11], dtype=np.int64),
              "model/per-user.values": np.array([1.0, 2.0, 3.0]), "model/per-user.entities": legacy}
    c = ck.Checkpointer(str(tmp_path))
    c.save(arrays, meta)
    st = c.load_cd()
    m = st["model"].get("per-user")
    assert list(m.entity_ids) == ids and np.array_equal(m.values, [1.0, 2.0, 3.0])
    c.save(arrays, dict(meta, format_version=ck.FORMAT_VERSION + 1))
    with pytest.raises(RuntimeError, match="format version"):
        c.load_cd()


@pytest.mark.parametrize("with_world_size", [True, False])
def test_versionless_length_prefixed_checkpoint_loads(tmp_path, with_world_size):
    """Builds between the two formats wrote length-prefixed id tables (and a world size) WITHOUT format_version;
    such files must not be decoded as newline-joined ids. Without the world size the table is sniffed."""
    from photon_ml_amd.utils import checkpoint as ck
    ids = ["u1", "a\nb", "ü"]
    meta = {"model": {"coordinates": [{"id": "per-user", "kind": "random", "shard": "s", "re_type": "userId",
                                       "task": "LINEAR_REGRESSION", "dim": 4, "n_entities": 3}]},
            "iteration": 1, "next": 0}
    if with_world_size:
        meta["world_size"] = 1
    arrays = {"model/per-user.keys": np.array([0, 5, 11], dtype=np.int64),
              "model/per-user.values": np.array([1.0, 2.0, 3.0]),
              "model/per-user.entities": ck._strings_to_array(ids)}
    c = ck.Checkpointer(str(tmp_path))
    c.save(arrays, meta)
    m = c.load_cd()["model"].get("per-user")
    assert list(m.entity_ids) == ids


def test_resume_with_down_sampling_draws_the_same_samples(tmp_path):
    """The down-sampling seed sequence position is part of the checkpoint: a run resumed in a fresh
    process trains its down-sampled fixed-effect updates on the same samples as an uninterrupted run."""
    from photon_ml_amd.sampling.samplers import reset_seed_sequence

    def setup():
        data, val, coords, evs = _setup(seed=7)
        cfg = GLMOptimizationConfiguration(OptimizerConfig("TRON", 30, 1e-9), RegularizationContext("L2"), 1.0, 0.5)
        coords["g"] = FixedEffectCoordinate("g", data, FixedEffectDataConfiguration("global"), cfg,
                                            "LOGISTIC_REGRESSION", device="cpu")
        return coords, val, evs

    reset_seed_sequence()
    coords, val, evs = setup()
    full_model, _ = CoordinateDescent(coords, None, val, evs).run(3)

    reset_seed_sequence()
    coords, val, evs = setup()
    calls = {"n": 0}

    def bomb(rec):
        calls["n"] += 1
        if calls["n"] == 4:   # after "g" of sweep 2 (its seed drawn), before "u"
            raise Interrupt()
    ck = Checkpointer(str(tmp_path), "cd")
    with pytest.raises(Interrupt):
        CoordinateDescent(coords, None, val, evs, event_callback=bomb).run(3, checkpointer=ck, tag="t")
    reset_seed_sequence()     # a fresh process starts the sequence from the beginning
    coords, val, evs = setup()
    model, _ = CoordinateDescent(coords, None, val, evs).run(3, checkpointer=Checkpointer(str(tmp_path), "cd"),
                                                            tag="t")
    torch.testing.assert_close(model.get("g").glm.coefficients.means, full_model.get("g").glm.coefficients.means,
                               rtol=0, atol=1e-10)
