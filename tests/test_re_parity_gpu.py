"""Direct fp64 parity of the PRODUCTION random-effect kernels against the CPU float64 TRON, entity by entity.

Every fused per-entity solver the GAME config-5 path runs is checked against ``optimization/tron.py`` (the
LIBLINEAR-semantics TRON of the reference, ``TRON.scala:80-340``) on ``TorchGLMData`` in float64, one entity at a
time on its own projected rows (``SingleNodeOptimizationProblem.scala:85-103``):

* ``lean_quad``  -- ``re_tron_lean_kernel`` with quad-padded rows (wide entities, >= 12 entries per row), the
  primal fused path (row space off);
* ``resident``   -- ``re_tron_res_kernel`` (register-resident, forced for every eligible entity);
* ``rs_K``       -- ``rs_tron_dpp_kernel`` row-space classes of K = 20 / 32 / 48 / 64 rows, shipped layouts;
* ``rs_big``     -- ``rs_tron_big_kernel`` (65 .. 128 dense rows);
* the row-space back-map ``w = X^T L^-T beta`` (``btrsv`` + ``rs_primal``) is what produces every row-space W
  compared here, and a foreign warm start exercises ``beta_from_primal`` (``L^-1 X w``).

Two regimes. (1) ITERATION-LIMITED (tolerance 0, 4 TRON iterations): both sides take exactly the same iterations,
and W must agree to 1e-9 relative -- only rounding separates them. (2) CONVERGED (tolerance 1e-8): identical
iteration counts and stop reasons per entity; W to 1e-6 relative, because TRON stops on "function values converged"
where the point reached is pinned only to ~sqrt(eps f / lambda_min) (see test_game_gpu.py,
test_fused_entity_tron_matches_pass_path).
"""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from photon_ml_amd.data.game_data import GameData

pytestmark = pytest.mark.gpu


def make_entities(sizes, d_pool, nnz_row, seed, dense_pool=False):
    """One random-effect shard: entity k has ``sizes[k]`` rows, ``nnz_row`` features per row from its own pool of
    ``d_pool`` global features (+ an intercept column); logistic labels from a per-entity ground truth."""
    rng = np.random.default_rng(seed)
    D = len(sizes) * d_pool + 1
    rows, cols, vals, ids, z = [], [], [], [], []
    r = 0
    for k, n in enumerate(sizes):
        wt = rng.normal(size=d_pool) * 0.5
        for _ in range(n):
            f = np.arange(d_pool) if dense_pool else np.sort(rng.choice(d_pool, size=nnz_row, replace=False))
            v = rng.normal(size=f.size)
            rows += [r] * (f.size + 1)
            cols += list(k * d_pool + f) + [D - 1]
            vals += list(v) + [1.0]
            z.append(float(v @ wt[f]) + 0.2 * np.sin(k))
            ids.append(k)
            r += 1
    x = sp.csr_matrix((vals, (rows, cols)), shape=(r, D))
    y = (rng.random(r) < 1 / (1 + np.exp(-np.array(z)))).astype(float)
    return GameData(y, {"user": x}, {"userId": np.array(ids)})


def cpu_tron(data, l2, tol, max_iter, offsets=None, w0=None):
    """Per entity, the CPU float64 TRON on the entity's rows restricted to its features (the INDEX_MAP projection):
    {entity id: (w over the global features, iterations, convergence reason)}."""
    from photon_ml_amd.data.matrix import LabeledData
    from photon_ml_amd.function.losses import LOGISTIC
    from photon_ml_amd.function.objective import GLMObjective
    from photon_ml_amd.ops.reference import TorchGLMData
    from photon_ml_amd.optimization.tron import TRON
    x = data.shards["user"].tocsr()
    ids = data.id_tags["userId"]
    off = np.zeros(data.n_rows) if offsets is None else offsets
    out = {}
    for e in np.unique(ids):
        r = np.nonzero(ids == e)[0]
        xe = x[r]
        feats = np.unique(xe.indices)
        xl = xe[:, feats]
        gd = TorchGLMData(LabeledData(xl, data.response[r], off[r], np.ones(len(r))), torch.device("cpu"))
        opt = TRON(tolerance=tol, max_iterations=max_iter, track_state=False)
        start = torch.zeros(len(feats), dtype=torch.float64) if w0 is None else \
            torch.from_numpy(np.ascontiguousarray(w0[e][feats]))
        w, _ = opt.optimize(GLMObjective(LOGISTIC, l2_weight=l2), gd, start)
        full = np.zeros(x.shape[1])
        full[feats] = w.numpy()
        out[e] = (full, int(opt.current.iter), opt.convergence_reason())
    return out


def gpu_fit(data, l2, tol, max_iter, monkeypatch, offsets=None, start=None):
    """The production coordinate on the GPU; returns ({entity: w}, {entity: iterations}, coordinate)."""
    from photon_ml_amd.algorithm.coordinates import RandomEffectCoordinate
    from photon_ml_amd.data.random_effect import RandomEffectDataConfiguration
    from photon_ml_amd.optimization.config import (GLMOptimizationConfiguration, OptimizerConfig,
                                                   RegularizationContext)
    cfg = GLMOptimizationConfiguration(OptimizerConfig("TRON", max_iter, tol), RegularizationContext("L2"), l2)
    c = RandomEffectCoordinate("u", data, RandomEffectDataConfiguration("userId", "user"), cfg,
                               "LOGISTIC_REGRESSION", device="cuda", layout="segmented")
    got = {}
    c._defer_stats = lambda it, rc, act, sec: got.update(it=it.cpu().numpy(), rc=rc.cpu().numpy())
    ps = None if offsets is None else torch.from_numpy(offsets)
    m = c.update_model(start if start is not None else c.initialize_model(), ps)
    m.materialize()
    W = {e: np.asarray(m.coefficients_of(e).means, dtype=np.float64) for e in m.entity_ids}
    its = {e: int(got["it"][i]) for i, e in enumerate(c.dataset.entity_ids)}
    return W, its, c, m


CASES = {
    # name: (sizes, d_pool, nnz_row, dense_pool, env, expected component)
    "lean_quad": ([90, 120, 150, 200, 260, 75] * 4, 300, 16, False, {"PML_RE_ROW_SPACE": "0"}, "lean"),
    "resident": ([90, 120, 150, 200, 260, 75] * 2, 300, 16, False, {"PML_RE_ROW_SPACE": "0"}, "resident"),
    "rs_20": ([20] * 40 + [17] * 10, 120, 12, False, {}, "rs"),
    "rs_32": ([32] * 30 + [25] * 10, 150, 12, False, {}, "rs"),
    "rs_48": ([48] * 25 + [41] * 8, 160, 14, False, {}, "rs"),
    "rs_64": ([64] * 20 + [57] * 6, 200, 16, False, {}, "rs"),
    "rs_big": ([80] * 10 + [100] * 6 + [128] * 4, 150, 0, True, {}, "rs_big"),
}


def _check_routing(c, kind):
    rs, fused, sub = c._comps
    assert sub is None
    if kind == "lean":
        assert rs is None and fused is not None and fused.quad and fused.res is None
        assert all(not h and dm <= 1024 for dm, _, h in fused.launches)
    elif kind == "resident":
        assert rs is None and fused is not None and fused.res is not None
    else:
        assert fused is None and rs is not None
        ns = [cl.n for cl in rs.classes]
        assert (max(ns) > 64) == (kind == "rs_big"), ns


@pytest.mark.parametrize("case", list(CASES))
def test_production_re_kernel_matches_cpu_tron_fp64(case, monkeypatch):
    import photon_ml_amd.optimization.entity_tron as et
    sizes, dp, nnz, dense, env, kind = CASES[case]
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setattr(et, "RESIDENT", "force" if kind == "resident" else "0")
    data = make_entities(sizes, dp, nnz, seed=len(case), dense_pool=dense)
    # (1) iteration-limited: tolerance 0, every entity runs exactly 4 TRON iterations on both sides
    W, its, c, _ = gpu_fit(data, 1.0, 0.0, 4, monkeypatch)
    _check_routing(c, kind)
    ref = cpu_tron(data, 1.0, 0.0, 4)
    for e, (w_ref, it_ref, _) in ref.items():
        assert its[e] == it_ref == 4, (e, its[e], it_ref)
        err = np.abs(W[e] - w_ref).max() / max(np.abs(w_ref).max(), 1e-300)
        assert err < 1e-9, (case, e, err)
    # (2) converged: the same iteration count and stop reason per entity
    W, its, c, m = gpu_fit(data, 1.0, 1e-8, 60, monkeypatch)
    ref = cpu_tron(data, 1.0, 1e-8, 60)
    for e, (w_ref, it_ref, _) in ref.items():
        assert its[e] == it_ref, (case, e, its[e], it_ref)
        err = np.abs(W[e] - w_ref).max() / max(np.abs(w_ref).max(), 1e-300)
        assert err < 1e-6, (case, e, err)
    # (3) warm start from a FOREIGN model (row space: beta = L^-1 X w through btrsv) with new offsets
    off = np.sin(np.arange(data.n_rows)) * 0.3
    w_half = {e: W[e] * 0.5 for e in W}
    from photon_ml_amd.models.game import RandomEffectModel
    keys = np.concatenate([int(i) * m.dim + np.nonzero(w_half[e])[0] for i, e in enumerate(m.entity_ids)])
    vals = np.concatenate([w_half[e][np.nonzero(w_half[e])[0]] for e in m.entity_ids])
    foreign = RandomEffectModel(m.random_effect_type, m.feature_shard_id, "LOGISTIC_REGRESSION", m.entity_ids, m.dim,
                                keys, vals)
    W2, its2, _, _ = gpu_fit(data, 1.0, 0.0, 4, monkeypatch, offsets=off, start=foreign)
    ref2 = cpu_tron(data, 1.0, 0.0, 4, offsets=off, w0=w_half)
    for e, (w_ref, it_ref, _) in ref2.items():
        assert its2[e] == it_ref
        err = np.abs(W2[e] - w_ref).max() / max(np.abs(w_ref).max(), 1e-300)
        assert err < 1e-9, (case, "foreign warm start", e, err)
    # (4) ... converged from that warm start: the tolerances scale with the ZERO point (Optimizer.scala); the lean
    # kernel bounds ||g(0)|| without a pass (exact pass only if a gradient norm reaches the bound) -- the same
    # iteration counts as the CPU TRON's exact zero state
    W3, its3, _, _ = gpu_fit(data, 1.0, 1e-8, 60, monkeypatch, offsets=off, start=foreign)
    ref3 = cpu_tron(data, 1.0, 1e-8, 60, offsets=off, w0=w_half)
    for e, (w_ref, it_ref, _) in ref3.items():
        assert its3[e] == it_ref, (case, "warm converged", e, its3[e], it_ref)
        err = np.abs(W3[e] - w_ref).max() / max(np.abs(w_ref).max(), 1e-300)
        assert err < 1e-6, (case, "warm converged", e, err)


def test_dense_bucket_quad_rows_longer_than_64_match_cpu_tron(monkeypatch):
    """DenseEntityTronBatch (dense size buckets: every padded row is a dense CSR row of d entries) with d > 64 and
    quad rows: each row is longer than the 64 entries one lane group covers per round, so the lean kernel's tail
    loop over further quads runs. Iteration-limited and converged fits match the CPU float64 TRON per entity."""
    import photon_ml_amd.algorithm.coordinates as co
    from photon_ml_amd.algorithm.coordinates import RandomEffectCoordinate
    from photon_ml_amd.data.random_effect import RandomEffectDataConfiguration
    from photon_ml_amd.optimization.config import (GLMOptimizationConfiguration, OptimizerConfig,
                                                   RegularizationContext)
    data = make_entities([80, 95, 70, 100] * 6, 100, 0, seed=3, dense_pool=True)
    real = co.random_effect_tracker_stats
    captured = {}

    def spy(it, rs, sec):
        captured["it"] = it.numpy().copy()
        return real(it, rs, sec)
    monkeypatch.setattr(co, "random_effect_tracker_stats", spy)
    for tol, max_iter, bound in ((0.0, 4, 1e-9), (1e-8, 60, 1e-6)):
        captured.clear()
        cfg = GLMOptimizationConfiguration(OptimizerConfig("TRON", max_iter, tol), RegularizationContext("L2"), 1.0)
        c = RandomEffectCoordinate("u", data, RandomEffectDataConfiguration("userId", "user"), cfg,
                                   "LOGISTIC_REGRESSION", device="cuda", layout="dense")
        m = c.update_model(c.initialize_model())
        fz = [c._dense_fused(b, bk, 0.0) for b, bk in enumerate(c.dataset.buckets)]
        assert all(f is not None and f.quad and f.d > 64 for f in fz)
        ents = np.concatenate([bk.entities for bk in c.dataset.buckets])
        its = {c.dataset.entity_ids[k]: int(captured["it"][i]) for i, k in enumerate(ents)}
        ref = cpu_tron(data, 1.0, tol, max_iter)
        for e, (w_ref, it_ref, _) in ref.items():
            assert its[e] == it_ref, (tol, e, its[e], it_ref)
            w = np.asarray(m.coefficients_of(e).means, dtype=np.float64)
            err = np.abs(w - w_ref).max() / max(np.abs(w_ref).max(), 1e-300)
            assert err < bound, (tol, e, err)


def test_row_space_classes_over_two_streams_match_one_stream(monkeypatch):
    """PML_RS_STREAMS=2 (size classes spread over a second stream, opt-in) solves exactly what the one-stream
    launch order solves: same kernels on the same inputs, so bitwise equal W and iteration counts; cold and warm
    (a warm start passes beta0, which the cold start leaves None: record_stream must skip it)."""
    from photon_ml_amd.optimization import row_space
    data = make_entities([20] * 30 + [32] * 20 + [48] * 12 + [64] * 8, 150, 12, seed=17)
    out = {}
    for ns in (1, 2):
        monkeypatch.setattr(row_space, "RS_STREAMS", ns)
        W, its, c, m = gpu_fit(data, 1.0, 1e-8, 30, monkeypatch)
        W2, its2, _, _ = gpu_fit(data, 1.0, 1e-8, 30, monkeypatch, offsets=np.cos(np.arange(data.n_rows)) * 0.2,
                                 start=m)
        out[ns] = (W, its, W2, its2)
    (a, ia, a2, ia2), (b, ib, b2, ib2) = out[1], out[2]
    assert ia == ib and ia2 == ib2
    for e in a:
        assert np.array_equal(np.asarray(a[e]), np.asarray(b[e])) and np.array_equal(np.asarray(a2[e]), np.asarray(b2[e]))
