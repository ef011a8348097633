"""GAME (fixed + random effects, coordinate descent) tests on CPU.

Mirrors photon-api/src/integTest/.../algorithm/*, model/*, data/RandomEffectDataSet tests and the CoordinateDescent
unit tests (photon-lib/src/test/.../algorithm/CoordinateDescentTest.scala)."""
from collections import OrderedDict

import numpy as np
import pytest
import torch

from photon_ml_amd.algorithm.coordinate_descent import CoordinateDescent
from photon_ml_amd.algorithm.coordinates import FixedEffectCoordinate, RandomEffectCoordinate
from photon_ml_amd.data.game_data import generate_game_data
from photon_ml_amd.data.random_effect import (FixedEffectDataConfiguration, RandomEffectDataConfiguration,
                                              RandomEffectDataset, reservoir_keys, java_string_hash)
from photon_ml_amd.evaluation.evaluators import build_evaluator
from photon_ml_amd.optimization.config import (GLMOptimizationConfiguration, OptimizerConfig, RegularizationContext)
from photon_ml_amd.projector import RandomProjection


def _cfg(opt="TRON", lam=1.0, it=30, tol=1e-8, reg="L2"):
    return GLMOptimizationConfiguration(OptimizerConfig(opt, it, tol), RegularizationContext(reg), lam)


def _coords(data, task="LINEAR_REGRESSION", re_opt="TRON"):
    return OrderedDict([
        ("global", FixedEffectCoordinate("global", data, FixedEffectDataConfiguration("global"), _cfg(), task,
                                         device="cpu")),
        ("per-user", RandomEffectCoordinate("per-user", data, RandomEffectDataConfiguration("userId", "user"),
                                            _cfg(re_opt), task, device="cpu")),
        ("per-item", RandomEffectCoordinate("per-item", data, RandomEffectDataConfiguration("itemId", "item"),
                                            _cfg(re_opt), task, device="cpu")),
    ])


def test_java_hash_and_reservoir_keys():
    assert java_string_hash("userId") == -836030906
    assert java_string_hash("") == 0
    k = reservoir_keys("userId", np.array([0, 1, 2, 12345678901]))
    assert k.dtype == np.int64 and len(set(k.tolist())) == 4


def test_game_linear_mixed_effects_improves_rmse():
    data, _ = generate_game_data(n_rows=3000, seed=3)
    val, _ = generate_game_data(n_rows=3000, seed=3)
    coords = _coords(data)
    rmse = build_evaluator("RMSE", val.response, val.offsets, val.weights)
    cd = CoordinateDescent(coords, build_evaluator("SQUARED_LOSS", data.response), val, [rmse])
    model, evals = cd.run(2)
    fe_only = CoordinateDescent(OrderedDict([("global", coords["global"])]), None, val, [rmse])
    _, evals_fe = fe_only.run(1)
    assert evals[0][1] < 0.8 * evals_fe[0][1], (evals, evals_fe)
    # training loss monotone over coordinate updates
    losses = [h["training_loss"] for h in cd.history]
    assert all(b <= a * (1 + 1e-9) for a, b in zip(losses, losses[1:]))


def test_single_coordinate_matches_glm():
    data, _ = generate_game_data(n_rows=1500, seed=4, task="LOGISTIC_REGRESSION")
    coord = FixedEffectCoordinate("g", data, FixedEffectDataConfiguration("global"), _cfg("LBFGS", 1.0, 100, 1e-10),
                                  "LOGISTIC_REGRESSION", device="cpu")
    model, _ = CoordinateDescent(OrderedDict(g=coord)).run(1)
    from photon_ml_amd.function.losses import LOGISTIC
    from photon_ml_amd.function.objective import GLMObjective
    from photon_ml_amd.ops.reference import TorchGLMData
    from photon_ml_amd.optimization import LBFGS
    w, _ = LBFGS(tolerance=1e-10).optimize(GLMObjective(LOGISTIC, 1.0), TorchGLMData(data.labeled("global")),
                                           torch.zeros(data.shards["global"].shape[1], dtype=torch.float64))
    assert torch.allclose(model.get("g").glm.coefficients.means, w, atol=1e-6)


@pytest.mark.parametrize("re_opt,reg", [("LBFGS", "L2"), ("LBFGS", "L1"), ("TRON", "L2")])
def test_random_effect_matches_per_entity_solves(re_opt, reg):
    data, _ = generate_game_data(n_rows=800, n_users=12, seed=5, task="LOGISTIC_REGRESSION")
    cfg = _cfg(re_opt, 0.5, 200, 1e-12, reg)
    coord = RandomEffectCoordinate("u", data, RandomEffectDataConfiguration("userId", "user"), cfg,
                                   "LOGISTIC_REGRESSION", device="cpu")
    m = coord.update_model(coord.initialize_model())
    from photon_ml_amd.data.matrix import LabeledData
    from photon_ml_amd.function.losses import LOGISTIC
    from photon_ml_amd.function.objective import GLMObjective
    from photon_ml_amd.ops.reference import TorchGLMData
    from photon_ml_amd.optimization import LBFGS, OWLQN
    x = data.shards["user"]
    for eid in m.entity_ids[:5]:
        rows = np.nonzero(data.id_tags["userId"] == eid)[0]
        ld = LabeledData(x[rows], data.response[rows])
        if reg == "L1":
            opt, obj = OWLQN(0.5, tolerance=1e-12, max_iterations=300), GLMObjective(LOGISTIC, 0.0)
        else:
            opt, obj = LBFGS(tolerance=1e-12, max_iterations=300), GLMObjective(LOGISTIC, 0.5)
        w, _ = opt.optimize(obj, TorchGLMData(ld), torch.zeros(x.shape[1], dtype=torch.float64))
        got = m.coefficients_of(eid).means
        assert torch.allclose(got, w, atol=2e-4), (eid, got, w)


def test_reservoir_cap_and_passive_data():
    data, _ = generate_game_data(n_rows=2000, n_users=10, seed=6)
    cfg = RandomEffectDataConfiguration("userId", "user", active_data_upper_bound=20, passive_data_lower_bound=5)
    ds = RandomEffectDataset(data, cfg)
    assert ds.n_active.max() <= 20
    counts = np.bincount(ds.sample_entity, minlength=ds.n_entities)
    capped = counts > 20
    # weights of capped entities multiplied by count/cap
    for b in ds.buckets:
        for i, e in enumerate(b.entities):
            if capped[e]:
                w = b.w[i][b.rows[i] >= 0]
                assert torch.allclose(w, torch.full_like(w, counts[e] / 20))
    assert len(ds.passive_rows) > 0
    assert not np.intersect1d(ds.passive_rows, ds.active_rows).size


def test_random_projection_and_feature_selection_run():
    data, _ = generate_game_data(n_rows=1000, n_users=8, d_user=12, seed=7)
    for cfg in (RandomEffectDataConfiguration("userId", "user", projector_type=RandomProjection(4)),
                RandomEffectDataConfiguration("userId", "user", features_to_samples_ratio=0.05)):
        coord = RandomEffectCoordinate("u", data, cfg, _cfg("TRON"), "LINEAR_REGRESSION", device="cpu")
        m = coord.update_model(coord.initialize_model())
        s = coord.score(m)
        assert torch.isfinite(s).all() and float(s.abs().sum()) > 0


@pytest.mark.parametrize("task,opt", [("LOGISTIC_REGRESSION", "TRON"), ("LINEAR_REGRESSION", "LBFGS"),
                                      ("POISSON_REGRESSION", "TRON")])
def test_segmented_re_layout_matches_dense(task, opt):
    """Block-diagonal (segmented) random-effect solve == dense bucketed batch solve, entity by entity."""
    data, _ = generate_game_data(n_rows=2500, n_users=30, seed=12, task=task)
    cfg = _cfg(opt, 1.0, 100, 1e-10)
    out, coords = {}, {}
    for layout in ("dense", "segmented"):
        c = RandomEffectCoordinate("u", data, RandomEffectDataConfiguration("userId", "user"), cfg, task,
                                   compute_variance=True, device="cpu", layout=layout)
        assert c.dataset.layout == layout
        out[layout] = c.update_model(c.initialize_model())
        coords[layout] = c
    a, b = out["dense"], out["segmented"]
    # fast device scoring of the just-solved model == generic model scoring
    assert torch.allclose(coords["segmented"].score(b), coords["dense"].score(a), atol=1e-6)
    assert torch.allclose(coords["segmented"].score(b), b.score(data, "cpu"), atol=1e-10)
    assert list(a.entity_ids) == list(b.entity_ids)
    for e in a.entity_ids:
        np.testing.assert_allclose(a.coefficients_of(e).means.numpy(), b.coefficients_of(e).means.numpy(),
                                   rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(a.coefficients_of(e).variances.numpy(), b.coefficients_of(e).variances.numpy(),
                                   rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("task", ["LOGISTIC_REGRESSION", "POISSON_REGRESSION", "LINEAR_REGRESSION"])
def test_fused_cg_step_matches_unfused_tron(task):
    """The fused per-entity CG iteration (one segmented kernel; CPU: same arithmetic in torch) gives the same
    block-diagonal TRON solution as the op-by-op vectorised CG."""
    from photon_ml_amd.function.losses import loss_for_task
    from photon_ml_amd.optimization.batched import batched_tron
    data, _ = generate_game_data(n_rows=2000, n_users=25, seed=5, task=task)
    c = RandomEffectCoordinate("u", data, RandomEffectDataConfiguration("userId", "user"), _cfg("TRON"), task,
                               device="cpu", layout="segmented")
    seg = c.dataset.seg
    loss = loss_for_task(task)
    W0 = torch.zeros(c.dataset.d_total, dtype=torch.float64)
    res = {f: batched_tron(seg, loss, 1.0, W0, 1e-9, 30, fused=f) for f in (False, True)}
    assert torch.equal(res[False].iters, res[True].iters)
    assert torch.allclose(res[False].W, res[True].W, rtol=1e-9, atol=1e-11)
    assert torch.allclose(res[False].f, res[True].f, rtol=1e-12)


@pytest.mark.parametrize("task,opt", [("LOGISTIC_REGRESSION", "TRON"), ("LINEAR_REGRESSION", "LBFGS"),
                                      ("POISSON_REGRESSION", "TRON"), ("LOGISTIC_REGRESSION", "LBFGS")])
def test_row_space_random_effect_solve_matches_primal(task, opt, monkeypatch):
    """Wide entities (n_e rows < d_e coefficients) solved in their row space (w = X^T L^-T beta, exact
    re-parametrisation) give the primal block-diagonal solution, the same per-entity iteration counts, and the
    same warm-started second coordinate-descent update; entities with more rows than coefficients, or beyond
    the row cap, stay on the primal path in the same solve."""
    # Zipf users: most have a few rows (wide -> row space), a few have many (-> primal path in the same solve)
    data, _ = generate_game_data(n_rows=2500, n_users=300, d_user=30, seed=21, task=task)
    cfg = _cfg(opt, 1.0, 60, 1e-10)
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("PML_RE_ROW_SPACE", mode)
        c = RandomEffectCoordinate("u", data, RandomEffectDataConfiguration("userId", "user"), cfg, task,
                                   device="cpu", layout="segmented")
        m1 = c.update_model(c.initialize_model())
        it1 = c.last_stats
        m2 = c.update_model(m1, partial_score=torch.from_numpy(np.sin(np.arange(data.n_rows)) * 0.3))
        out[mode] = (c, m1, m2, it1)
        if mode == "1":
            assert c._rs is not None and 0 < c._rs.B < int((c.dataset.n_active > 0).sum())
            # Zipf sizes: several size classes, each padded to its own largest entity
            ns = [k.n for k in c._rs.classes]
            assert len(ns) > 1 and ns == sorted(ns) and c._rs.size == sum(k.B * k.n for k in c._rs.classes)
    (c0, a1, a2, s0), (c1, b1, b2, s1) = out["0"], out["1"]
    # same iterates in exact arithmetic; at tol 1e-10 rounding can move a convergence test by one iteration
    assert s0["mean_iterations"] == pytest.approx(s1["mean_iterations"], rel=0.02)
    # entities that stop on "objective not improving" may stop one rounding-level step apart
    for (a, b), tol in (((a1, b1), 2e-7), ((a2, b2), 5e-6)):
        for e in a.entity_ids:
            np.testing.assert_allclose(a.coefficients_of(e).means.numpy(), b.coefficients_of(e).means.numpy(),
                                       rtol=1e-4, atol=tol)
    assert torch.allclose(c0.score(a2), c1.score(b2), atol=1e-5)


def test_row_space_lazy_primal_model(monkeypatch):
    """When every entity is solved in its row space, the returned model defers w = X^T L^-T beta until it is
    read: scores (L beta), the regularization term (||beta||^2) and the warm-started next update need no
    transpose pass, and the materialised coefficients equal the eager ones."""
    data, _ = generate_game_data(n_rows=600, n_items=200, d_item=40, seed=31, task="LOGISTIC_REGRESSION")
    cfg = _cfg("TRON", 1.0, 60, 1e-10)
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("PML_RE_LAZY_PRIMAL", mode)
        c = RandomEffectCoordinate("i", data, RandomEffectDataConfiguration("itemId", "item"), cfg,
                                   "LOGISTIC_REGRESSION", device="cpu", layout="segmented")
        m1 = c.update_model(c.initialize_model())
        s1, r1 = c.score(m1), c.regularization_term_value(m1)
        m2 = c.update_model(m1, partial_score=torch.from_numpy(np.cos(np.arange(data.n_rows)) * 0.3))
        s2, r2 = c.score(m2), c.regularization_term_value(m2)
        out[mode] = (m1, m2, s1, s2, r1, r2, m2.materialized)
    (a1, a2, as1, as2, ar1, ar2, amat), (b1, b2, bs1, bs2, br1, br2, bmat) = out["0"], out["1"]
    assert amat and not bmat            # lazy path taken (all entities in row space), eager path materialised
    torch.testing.assert_close(as1, bs1, rtol=1e-9, atol=1e-10)
    torch.testing.assert_close(as2, bs2, rtol=1e-9, atol=1e-10)
    assert ar1 == pytest.approx(br1, rel=1e-9) and ar2 == pytest.approx(br2, rel=1e-9)
    np.testing.assert_allclose(b2.values, a2.values, rtol=1e-8, atol=1e-10)
    assert b2.materialized


@pytest.mark.parametrize("layout", ["dense", "segmented"])
def test_random_effect_reused_coordinate_starts_from_given_model(layout):
    """A coordinate reused across configurations (GameEstimator.fit) must start from the model it is GIVEN, not
    from the solver state of its previous solve: a zero initial model after a solve == a fresh coordinate."""
    data, _ = generate_game_data(n_rows=1200, n_users=40, d_user=8, seed=41, task="LOGISTIC_REGRESSION")
    cfg1, cfg2 = _cfg("TRON", 0.3, 2, 1e-12), _cfg("TRON", 3.0, 2, 1e-12)
    dc = RandomEffectDataConfiguration("userId", "user")
    reused = RandomEffectCoordinate("u", data, dc, cfg1, "LOGISTIC_REGRESSION", device="cpu", layout=layout)
    reused.update_model(reused.initialize_model())
    reused.set_config(cfg2)
    got = reused.update_model(reused.initialize_model())
    fresh = RandomEffectCoordinate("u", data, dc, cfg2, "LOGISTIC_REGRESSION", device="cpu", layout=layout)
    want = fresh.update_model(fresh.initialize_model())
    for e in want.entity_ids:
        np.testing.assert_allclose(got.coefficients_of(e).means.numpy(), want.coefficients_of(e).means.numpy(),
                                   rtol=1e-10, atol=1e-12)
    # the coordinate's own last model still warm-starts from the cached state (same result as mapping it)
    again = reused.update_model(got)
    mapped = fresh.update_model(want)
    for e in want.entity_ids:
        np.testing.assert_allclose(again.coefficients_of(e).means.numpy(), mapped.coefficients_of(e).means.numpy(),
                                   rtol=1e-6, atol=1e-8)


def test_estimator_without_warm_start_matches_fresh_fit():
    from photon_ml_amd.estimators.game_estimator import GameEstimator
    data, _ = generate_game_data(n_rows=1500, n_users=30, seed=42, task="LOGISTIC_REGRESSION")
    dcs = OrderedDict([("global", FixedEffectDataConfiguration("global")),
                       ("per-user", RandomEffectDataConfiguration("userId", "user"))])
    cfgs = [{"global": _cfg("LBFGS", lam, 5, 1e-12), "per-user": _cfg("TRON", lam, 3, 1e-12)} for lam in (0.1, 5.0)]

    def fit(cs):
        est = (GameEstimator(device="cpu").set_training_task("LOGISTIC_REGRESSION")
               .set_coordinate_data_configurations(dcs).set_coordinate_descent_iterations(2).set_warm_start(False))
        return est.fit(data, None, cs)

    both, alone = fit(cfgs), fit(cfgs[1:])
    a, b = both[1].model, alone[0].model
    torch.testing.assert_close(a.get("global").glm.coefficients.means, b.get("global").glm.coefficients.means,
                               rtol=1e-9, atol=1e-11)
    for e in b.get("per-user").entity_ids:
        np.testing.assert_allclose(a.get("per-user").coefficients_of(e).means.numpy(),
                                   b.get("per-user").coefficients_of(e).means.numpy(), rtol=1e-9, atol=1e-11)


def test_device_build_keys_match_host():
    from photon_ml_amd.data.re_build import reservoir_keys_t
    uids = np.array([0, 1, 2, 12345678901, -5, 2 ** 62 + 17, -(2 ** 62)], dtype=np.int64)
    for t in ("userId", "songId", ""):
        host = reservoir_keys(t, uids)
        dev = reservoir_keys_t(java_string_hash(t), torch.from_numpy(uids)).numpy()
        assert np.array_equal(host, dev), (t, host, dev)


@pytest.mark.parametrize("cap,passive,ratio", [(20, 5, None), (7, 0, 0.05), (None, None, 0.3), (3, 2, 0.5)])
def test_random_effect_device_build_matches_host(cap, passive, ratio, monkeypatch):
    """K21 reservoir, passive set and K13 Pearson selection as whole-coordinate sorts / segment sums
    (data/re_build.py) == the host implementation: same active / passive rows, weights and selected features."""
    data, _ = generate_game_data(n_rows=3000, n_users=25, d_user=20, seed=44, task="LOGISTIC_REGRESSION")
    cfg = RandomEffectDataConfiguration("userId", "user", active_data_upper_bound=cap,
                                        passive_data_lower_bound=passive, features_to_samples_ratio=ratio)
    out = {}
    for mode in ("0", "force"):
        monkeypatch.setenv("PML_RE_DEVICE_BUILD", mode)
        ds = RandomEffectDataset(data, cfg, "cpu", layout="dense")
        assert ds.device_build == (mode == "force")
        out[mode] = ds
    a, b = out["0"], out["force"]
    assert np.array_equal(a.active_rows, b.active_rows) and np.array_equal(a.passive_rows, b.passive_rows)
    np.testing.assert_array_equal(a.weight_mult, b.weight_mult)
    xa, xb = a.x_active.tocsr(), b.x_active.tocsr()
    xa.sort_indices()
    xb.sort_indices()
    assert np.array_equal(xa.indptr, xb.indptr) and np.array_equal(xa.indices, xb.indices)
    np.testing.assert_array_equal(xa.data, xb.data)


@pytest.mark.parametrize("opt", ["TRON", "LBFGS"])
def test_primal_entity_subset_matches_frozen_full_problem(opt, monkeypatch):
    """Entities outside the row-space batch are solved on their own rows / coefficients (entity_subset) — same
    coefficients, scores and iteration counts as the frozen-mask solve over the whole block-diagonal problem."""
    data, _ = generate_game_data(n_rows=3000, n_users=300, d_user=30, seed=46, task="LOGISTIC_REGRESSION")
    cfg = _cfg(opt, 1.0, 40, 1e-10)
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("PML_RE_PRIMAL_SUBSET", mode)
        c = RandomEffectCoordinate("u", data, RandomEffectDataConfiguration("userId", "user"), cfg,
                                   "LOGISTIC_REGRESSION", device="cpu", layout="segmented")
        m1 = c.update_model(c.initialize_model())
        m2 = c.update_model(m1, partial_score=torch.from_numpy(np.cos(np.arange(data.n_rows)) * 0.2))
        out[mode] = (c, m2, c.last_stats)
        assert (getattr(c, "_sub", None) is not None) == (mode == "1")
    (c0, a, s0), (c1, b, s1) = out["0"], out["1"]
    assert 0 < c1._rs.B < int((c1.dataset.n_active > 0).sum())
    assert s0["mean_iterations"] == pytest.approx(s1["mean_iterations"], rel=1e-6)
    for e in a.entity_ids:
        np.testing.assert_allclose(b.coefficients_of(e).means.numpy(), a.coefficients_of(e).means.numpy(),
                                   rtol=1e-8, atol=1e-10)
    torch.testing.assert_close(c1.score(b), c0.score(a), rtol=1e-8, atol=1e-10)


def test_canonical_csr_check():
    """The per-entity Gram kernel needs strictly increasing columns inside each row (row starts may drop)."""
    from photon_ml_amd.optimization.row_space import _canonical_csr
    nip = torch.tensor([0, 2, 2, 5, 6])
    good = torch.tensor([3, 7, 1, 4, 9, 0])
    assert _canonical_csr((nip, good, torch.ones(6)), torch.device("cpu")) is not None
    dup = torch.tensor([3, 7, 1, 4, 4, 0])
    assert _canonical_csr((nip, dup, torch.ones(6)), torch.device("cpu")) is None
    assert _canonical_csr(None, torch.device("cpu")) is None


@pytest.mark.parametrize("trans", [False, True])
def test_batched_trsv_host_path(trans):
    """batched_trsv on the host (torch's triangular solve; the device runs btrsv_kernel): L y = x / L^T y = x for a
    batch of Cholesky factors, the row-space back-map's and warm-start projection's only use of the factors."""
    from photon_ml_amd.ops.native import batched_trsv
    g = torch.Generator().manual_seed(3 + trans)
    A = torch.randn(17, 9, 12, dtype=torch.float64, generator=g)
    L = torch.linalg.cholesky(A @ A.transpose(1, 2))
    x = torch.randn(17, 9, dtype=torch.float64, generator=g)
    y = batched_trsv(L, x, trans)
    M = L.transpose(1, 2) if trans else L
    torch.testing.assert_close(torch.bmm(M, y.unsqueeze(-1)).squeeze(-1), x, rtol=1e-10, atol=1e-10)
    torch.testing.assert_close(y, torch.bmm(torch.linalg.inv(M), x.unsqueeze(-1)).squeeze(-1), rtol=1e-9,
                               atol=1e-9)
    out = torch.full_like(x, float("nan"))
    assert batched_trsv(L, x, trans, out=out) is out and torch.equal(out, y)


def test_lazy_glm_data_builds_once_on_first_use():
    """LazyGLMData (the random-effect pass layout built on first use): no build until an attribute is read, then
    exactly one build, every later access delegated to the built object."""
    from photon_ml_amd.data.random_effect import LazyGLMData
    calls = []

    class Backend:
        n_rows = 7

        def matvec(self, w):
            return w * 2

    def build():
        calls.append(1)
        return Backend()

    lazy = LazyGLMData(build)
    assert not lazy.built and calls == []
    assert lazy.n_rows == 7 and lazy.built and calls == [1]
    assert lazy.matvec(3) == 6 and calls == [1]
    with pytest.raises(AttributeError):
        lazy.no_such_attribute
    assert calls == [1]


def test_prefetch_shard_is_a_no_op_off_the_gpu():
    """GameData.prefetch_shard copies a host shard to a GPU in the background; on the CPU (or for an unknown /
    device-resident shard) it does nothing and take_prefetched hands back nothing."""
    data = generate_game_data(n_rows=200, seed=5)
    data = data[0] if isinstance(data, tuple) else data
    sid = next(iter(data.shards))
    assert data.prefetch_shard(sid, "cpu") is False
    assert data.take_prefetched(sid, data.shard(sid)) is None
