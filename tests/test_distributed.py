"""Multi-process data/entity parallelism on CPU (gloo, world sizes 2, 4 and 8 — the 8-GPU node rehearsed with one
process per rank) vs single-process results.

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


WORLDS = [2, 4, 8]


@pytest.mark.parametrize("world", WORLDS)
def test_sharding_primitives(tmp_path, world):
    _launch("sharding", tmp_path, world=world)
    n = [int(np.load(tmp_path / f"shard_r{r}.npy")[0]) for r in range(world)]
    assert sum(n) == 80 * world
    perms = [np.load(tmp_path / f"perm_r{r}.npy") for r in range(world)]
    for p in perms[1:]:
        assert np.array_equal(perms[0], p)


@pytest.mark.parametrize("world", WORLDS)
def test_data_parallel_glm_matches_single_process(tmp_path, world):
    _launch("glm", tmp_path, world=world)
    from photon_ml_amd.data.synthetic import generate_glm_data
    from photon_ml_amd.estimators.game_estimator import train_generalized_linear_model
    from photon_ml_amd.optimization.config import RegularizationContext
    data, _ = generate_glm_data("LOGISTIC_REGRESSION", 3000, 40, density=0.2, seed=7)
    for opt, reg in (("LBFGS", "L2"), ("TRON", "L2"), ("LBFGS", "L1")):
        ref = train_generalized_linear_model(data, "LOGISTIC_REGRESSION", opt, RegularizationContext(reg), [1.0],
                                             max_iterations=200, tolerance=1e-10, device="cpu")[0][1]
        ws = [np.load(tmp_path / f"glm_{opt}_{reg}_r{r}.npy") for r in range(world)]
        for w in ws[1:]:
            assert np.array_equal(ws[0], w)  # replicated optimizer: bitwise identical on every rank
        np.testing.assert_allclose(ws[0], ref.coefficients.means.numpy(), rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_feature_sharded_optimizer_matches_single_process(tmp_path, world):
    """Optimizer state sharded over features (all-gather w / reduce-scatter g / sharded L-BFGS history with the
    vector-free two-loop) reproduces the replicated single-process optimum for L-BFGS, TRON, OWL-QN and a
    standardized problem; 3 and 8 ranks exercise uneven feature slices (41 = 14 + 14 + 13, 41 = 6 + 5 x 7)."""
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


@pytest.mark.parametrize("world", WORLDS)
def test_entity_sharded_game_matches_single_process(tmp_path, world):
    _launch("game", tmp_path, world=world)
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
    fes = [np.load(tmp_path / f"game_fe_r{r}.npy") for r in range(world)]
    for fe in fes[1:]:
        assert np.array_equal(fes[0], fe)
    np.testing.assert_allclose(fes[0], ref.model.get("global").glm.coefficients.means.numpy(), rtol=1e-5,
                               atol=1e-6)
    evs = [np.load(tmp_path / f"game_eval_r{r}.npy") for r in range(world)]
    for ev in evs[1:]:
        assert np.allclose(evs[0], ev)
    # AUC, LOGISTIC_LOSS and the per-user AUC:userId (entity-grouped, across ranks)
    np.testing.assert_allclose(evs[0], [v for _, v in ref.evaluations], rtol=1e-6)
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


@pytest.mark.parametrize("world", WORLDS)
def test_entity_placement_makes_primary_coordinate_route_free(tmp_path, world):
    """Rows placed on their primary-entity owners at ingest: the primary random-effect coordinate reproduces the
    per-update-routed one bitwise (same rows in the same order on the owner) and moves zero bytes per update; the
    other random-effect coordinate still routes; whole fits with and without placement agree."""
    _launch("placed", tmp_path, world=world)
    # routed scores come back to the rows' source ranks, placed ones stay on the owners: compare per uid
    cat = lambda kind: (lambda a: a[np.argsort(a[:, 0])])(
        np.concatenate([np.load(tmp_path / f"{kind}_scores_r{r}.npy") for r in range(world)]))
    a, b = cat("routed"), cat("placed")
    assert a.shape == b.shape == (2400, 2) and np.array_equal(a, b)
    for r in range(world):
        nb = np.load(tmp_path / f"fit_auto_bytes_r{r}.npy")
        assert nb[0] == 0 and nb[1] > 0
        assert np.load(tmp_path / f"fit_none_bytes_r{r}.npy")[0] > 0
    fas = [np.load(tmp_path / f"fit_auto_fe_r{r}.npy") for r in range(world)]
    for fa in fas[1:]:
        assert np.array_equal(fas[0], fa)
    fa0 = fas[0]
    # the fixed effect sums its per-rank gradients over other row sets: equal to rounding
    np.testing.assert_allclose(fa0, np.load(tmp_path / "fit_none_fe_r0.npy"), rtol=1e-7, atol=1e-9)


@pytest.mark.parametrize("world", [4, 8])
def test_ranks_without_entities_of_a_type(tmp_path, world):
    """A random-effect type with 2 entities on 4 / 8 ranks: most ranks own none of it (LPT bin packing leaves them
    empty). Training, the AUC:regionId evaluator and the per-rank model parts still match the single process."""
    _launch("sparse_re", tmp_path, world=world)
    sys.path.insert(0, HERE)
    from dist_worker import sparse_re_data, sparse_re_estimator
    from photon_ml_amd.io.index_map import DefaultIndexMap
    from photon_ml_amd.io.model_io import load_game_model
    from photon_ml_amd.optimization.config import (GLMOptimizationConfiguration, OptimizerConfig,
                                                   RegularizationContext)
    owned = [int(np.load(tmp_path / f"sparse_owned_r{r}.npy")[0]) for r in range(world)]
    assert sum(owned) == 2 and owned.count(0) >= world - 2, owned
    data = sparse_re_data()
    tr, va = data.subset(np.arange(2400)), data.subset(np.arange(2400, 3000))
    cfg = GLMOptimizationConfiguration(OptimizerConfig("TRON", 50, 1e-10), RegularizationContext("L2"), 1.0)
    ref = sparse_re_estimator().fit(tr, va, [{"global": cfg, "per-user": cfg, "per-region": cfg}])[0]
    fes = [np.load(tmp_path / f"sparse_fe_r{r}.npy") for r in range(world)]
    for fe in fes[1:]:
        assert np.array_equal(fes[0], fe)
    np.testing.assert_allclose(fes[0], ref.model.get("global").glm.coefficients.means.numpy(), rtol=1e-5,
                               atol=1e-6)
    np.testing.assert_allclose(np.load(tmp_path / "sparse_eval_r0.npy"), [v for _, v in ref.evaluations],
                               rtol=1e-6)
    maps = {s: DefaultIndexMap.from_keys([f"f{j}\u0001t" for j in range(data.shards[s].shape[1])])
            for s in data.shards}
    loaded = load_game_model(str(tmp_path / "model"), maps)
    a, b = loaded.get("per-region"), ref.model.get("per-region")
    assert sorted(a.entity_ids) == sorted(b.entity_ids) and len(b.entity_ids) == 2
    for e in b.entity_ids:
        ca, cb = a.coefficients_of(e).means.numpy(), b.coefficients_of(e).means.numpy()
        keep = np.abs(cb) > 1e-4
        np.testing.assert_allclose(ca[keep], cb[keep], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("world", [2, 3])
def test_chunked_all_to_all_matches_one_collective(tmp_path, world):
    """The device all-to-all in rounds of bounded size (RowRouter._a2a_device: one multi-GB RCCL call left the
    output's tail unwritten) reproduces the single collective exactly, for uneven and empty segments."""
    _launch("a2a", tmp_path, world=world)
    assert all((tmp_path / f"a2a_r{r}.npy").exists() for r in range(world))
