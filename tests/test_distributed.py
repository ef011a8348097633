"""Multi-process data/entity parallelism on CPU (gloo, world_size 2) vs single-process results.

Mirrors the reference's distributed-vs-local equivalence tests (DistributedObjectiveFunctionTest with several
partitions, GameEstimatorIntegTest) using real process groups: row-sharded fixed effects with one packed
all-reduce per evaluation, entity-sharded random effects with all-to-all residual routing.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(kind, out, world=2, timeout=600, **env_extra):
    port = _free_port()
    env = dict(os.environ, PML_BACKEND="torch", OMP_NUM_THREADS="2", **env_extra)
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"), kind, str(r), str(world),
                               str(port), str(out)], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for r in range(world)]
    outs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(o.decode(errors="replace"))
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-4000:]


def test_sharding_primitives(tmp_path):
    _launch("sharding", tmp_path)
    n = [int(np.load(tmp_path / f"shard_r{r}.npy")[0]) for r in range(2)]
    assert sum(n) == 160
    p0, p1 = np.load(tmp_path / "perm_r0.npy"), np.load(tmp_path / "perm_r1.npy")
    assert np.array_equal(p0, p1)


def test_data_parallel_glm_matches_single_process(tmp_path):
    _launch("glm", tmp_path)
    from photon_ml_amd.data.synthetic import generate_glm_data
    from photon_ml_amd.estimators.game_estimator import train_generalized_linear_model
    from photon_ml_amd.optimization.config import RegularizationContext
    data, _ = generate_glm_data("LOGISTIC_REGRESSION", 3000, 40, density=0.2, seed=7)
    for opt, reg in (("LBFGS", "L2"), ("TRON", "L2"), ("LBFGS", "L1")):
        ref = train_generalized_linear_model(data, "LOGISTIC_REGRESSION", opt, RegularizationContext(reg), [1.0],
                                             max_iterations=200, tolerance=1e-10, device="cpu")[0][1]
        w0 = np.load(tmp_path / f"glm_{opt}_{reg}_r0.npy")
        w1 = np.load(tmp_path / f"glm_{opt}_{reg}_r1.npy")
        assert np.array_equal(w0, w1)  # replicated optimizer: bitwise identical on every rank
        np.testing.assert_allclose(w0, ref.coefficients.means.numpy(), rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("world", [2, 3])
def test_feature_sharded_optimizer_matches_single_process(tmp_path, world):
    """Optimizer state sharded over features (all-gather w / reduce-scatter g / sharded L-BFGS history with the
    vector-free two-loop) reproduces the replicated single-process optimum for L-BFGS, TRON, OWL-QN and a
    standardized problem; 3 ranks exercise uneven feature slices (41 = 14 + 14 + 13)."""
    _launch("fsdp", tmp_path, world=world)
    from photon_ml_amd.data.synthetic import generate_glm_data
    from photon_ml_amd.estimators.game_estimator import train_generalized_linear_model
    from photon_ml_amd.normalization.context import NormalizationContext
    from photon_ml_amd.optimization.config import RegularizationContext
    from photon_ml_amd.stat.summary import BasicStatisticalSummary
    data, _ = generate_glm_data("LOGISTIC_REGRESSION", 3000, 41, density=0.2, seed=7)
    for opt, reg, norm in (("LBFGS", "L2", None), ("TRON", "L2", None), ("LBFGS", "L1", None),
                           ("LBFGS", "L2", "STANDARDIZATION")):
        nc = None
        if norm:
            nc = NormalizationContext.build(norm, BasicStatisticalSummary.compute(data.x), data.n_features - 1)
        ref = train_generalized_linear_model(data, "LOGISTIC_REGRESSION", opt, RegularizationContext(reg), [1.0],
                                             normalization=nc, max_iterations=200, tolerance=1e-10,
                                             device="cpu")[0][1]
        ws = [np.load(tmp_path / f"fsdp_{opt}_{reg}_{norm}_r{r}.npy") for r in range(world)]
        for w in ws[1:]:
            assert np.array_equal(ws[0], w)  # every rank gathers the same model
        np.testing.assert_allclose(ws[0], ref.coefficients.means.numpy(), rtol=1e-5, atol=1e-6)
    # estimator API path (ModelTraining with feature_sharded=True) incl. Hessian-diagonal variances
    ref = train_generalized_linear_model(data, "LOGISTIC_REGRESSION", "TRON", RegularizationContext("L2"), [1.0],
                                         max_iterations=100, tolerance=1e-10, compute_variance=True,
                                         device="cpu")[0][1]
    api = np.load(tmp_path / "fsdp_api_r0.npy")
    np.testing.assert_allclose(api[0], ref.coefficients.means.numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(api[1], ref.coefficients.variances.numpy(), rtol=1e-5)


def test_entity_sharded_game_matches_single_process(tmp_path):
    _launch("game", tmp_path)
    from photon_ml_amd.data.game_data import generate_game_data
    from photon_ml_amd.data.random_effect import FixedEffectDataConfiguration, RandomEffectDataConfiguration
    from photon_ml_amd.estimators.game_estimator import GameEstimator
    from photon_ml_amd.io.index_map import DefaultIndexMap
    from photon_ml_amd.io.model_io import load_game_model
    from photon_ml_amd.optimization.config import (GLMOptimizationConfiguration, OptimizerConfig,
                                                   RegularizationContext)
    data, _ = generate_game_data(n_rows=3000, n_users=40, n_items=25, seed=31, task="LOGISTIC_REGRESSION")
    tr, va = data.subset(np.arange(2400)), data.subset(np.arange(2400, 3000))
    cfg = GLMOptimizationConfiguration(OptimizerConfig("TRON", 50, 1e-10), RegularizationContext("L2"), 1.0)
    est = (GameEstimator(device="cpu").set_training_task("LOGISTIC_REGRESSION")
           .set_coordinate_data_configurations({"global": FixedEffectDataConfiguration("global"),
                                                "per-user": RandomEffectDataConfiguration("userId", "user"),
                                                "per-item": RandomEffectDataConfiguration("itemId", "item")})
           .set_coordinate_update_sequence(["global", "per-user", "per-item"])
           .set_coordinate_descent_iterations(2)
           .set_validation_evaluators(["AUC", "LOGISTIC_LOSS", "AUC:userId"]))
    ref = est.fit(tr, va, [{"global": cfg, "per-user": cfg, "per-item": cfg}])[0]
    fe0, fe1 = np.load(tmp_path / "game_fe_r0.npy"), np.load(tmp_path / "game_fe_r1.npy")
    assert np.array_equal(fe0, fe1)
    np.testing.assert_allclose(fe0, ref.model.get("global").glm.coefficients.means.numpy(), rtol=1e-5, atol=1e-6)
    ev0, ev1 = np.load(tmp_path / "game_eval_r0.npy"), np.load(tmp_path / "game_eval_r1.npy")
    assert np.allclose(ev0, ev1)
    np.testing.assert_allclose(ev0, [v for _, v in ref.evaluations], rtol=1e-6)
    # the per-rank model parts load back into one model equal to the single-process one
    maps = {s: DefaultIndexMap.from_keys([f"f{j}\u0001t" for j in range(data.shards[s].shape[1])])
            for s in data.shards}
    loaded = load_game_model(str(tmp_path / "model"), maps)
    for cid in ("per-user", "per-item"):
        a, b = loaded.get(cid), ref.model.get(cid)
        assert sorted(a.entity_ids) == sorted(b.entity_ids)
        for e in b.entity_ids[:10]:
            ca, cb = a.coefficients_of(e).means.numpy(), b.coefficients_of(e).means.numpy()
            keep = np.abs(cb) > 1e-4  # the Avro writer drops |w| <= 1e-4
            np.testing.assert_allclose(ca[keep], cb[keep], rtol=1e-5, atol=1e-6)


def test_forced_one_rank_group_is_bitwise_single_process(tmp_path):
    """PML_FORCE_DIST=1 with WORLD_SIZE=1: the entity-sharded GAME path (routing all-to-alls, distributed
    evaluators, per-rank model parts) runs through a one-rank process group — the mode the GPU test
    ``test_rccl_gpu.py`` uses to execute the RCCL code paths on a single MI355X. It must give the single-process
    model exactly (the distributed evaluators reduce in another order: 1e-12)."""
    for mode, flag in (("forced", "1"), ("plain", "0")):
        (tmp_path / mode).mkdir()
        _launch("game", tmp_path / mode, world=1, PML_FORCE_DIST=flag)
    assert np.array_equal(np.load(tmp_path / "forced/game_fe_r0.npy"), np.load(tmp_path / "plain/game_fe_r0.npy"))
    np.testing.assert_allclose(np.load(tmp_path / "forced/game_eval_r0.npy"),
                               np.load(tmp_path / "plain/game_eval_r0.npy"), rtol=1e-12)


def test_entity_placement_makes_primary_coordinate_route_free(tmp_path):
    """Rows placed on their primary-entity owners at ingest: the primary random-effect coordinate reproduces the
    per-update-routed one bitwise (same rows in the same order on the owner) and moves zero bytes per update; the
    other random-effect coordinate still routes; whole fits with and without placement agree."""
    _launch("placed", tmp_path)
    # routed scores come back to the rows' source ranks, placed ones stay on the owners: compare per uid
    cat = lambda kind: (lambda a: a[np.argsort(a[:, 0])])(
        np.concatenate([np.load(tmp_path / f"{kind}_scores_r{r}.npy") for r in range(2)]))
    a, b = cat("routed"), cat("placed")
    assert a.shape == b.shape == (2400, 2) and np.array_equal(a, b)
    for r in range(2):
        nb = np.load(tmp_path / f"fit_auto_bytes_r{r}.npy")
        assert nb[0] == 0 and nb[1] > 0
        assert np.load(tmp_path / f"fit_none_bytes_r{r}.npy")[0] > 0
    fa0, fa1 = np.load(tmp_path / "fit_auto_fe_r0.npy"), np.load(tmp_path / "fit_auto_fe_r1.npy")
    assert np.array_equal(fa0, fa1)
    # the fixed effect sums its per-rank gradients over other row sets: equal to rounding
    np.testing.assert_allclose(fa0, np.load(tmp_path / "fit_none_fe_r0.npy"), rtol=1e-7, atol=1e-9)
