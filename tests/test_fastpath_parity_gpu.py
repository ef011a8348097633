"""Default-on fast paths run both ways on the GPU and compared BITWISE (``torch.equal``) with the code they replace:
the fused line-search finish (``ls_finish_fused`` + ``ls_step_grad``), the fused offset update
(``DeviceGLMData.set_offsets_sum`` / ``offset_update_kernel``), the one-launch coefficient gather + cast
(``perm_cast`` in ``DeviceGLMData._vec``), the random-effect side-stream overlap (``PML_RE_OVERLAP``), the deferred
error check of the register-resident launch, and the device CSR router (``RowRouter.forward_csr_device``)."""
import numpy as np
import pytest
import torch

from photon_ml_amd.data.game_data import generate_game_data
from photon_ml_amd.data.synthetic import generate_glm_data
from photon_ml_amd.function.losses import LOGISTIC, POISSON
from photon_ml_amd.function.objective import GLMObjective

pytestmark = pytest.mark.gpu


def _dev_data(precision="f64", n=20000, d=3000, seed=5, task="LOGISTIC_REGRESSION"):
    from photon_ml_amd.ops.device import DeviceGLMData
    data, _ = generate_glm_data(task, n, d, density=0.01, seed=seed)
    return data, DeviceGLMData.from_labeled(data, "cuda", precision)


@pytest.mark.parametrize("precision", ["f64", "bf16"])
@pytest.mark.parametrize("loss", [LOGISTIC, POISSON])
def test_fused_line_search_finish_is_bitwise_the_unfused_path(precision, loss):
    """L-BFGS with the fused finish (step + transpose pass + gradient epilogue in one launch after the pass) vs
    the unfused finish (torch step, ``ls_finish_device``, torch epilogue): identical iterates, values, gradients."""
    from photon_ml_amd.optimization.lbfgs import LBFGS
    task = "LOGISTIC_REGRESSION" if loss is LOGISTIC else "POISSON_REGRESSION"
    out = []
    for fused in (True, False):
        _, dev = _dev_data(precision, task=task)
        if not fused:
            dev.ls_finish_fused = None           # MarginLineSearch.finish falls back to the unfused path
        obj = GLMObjective(loss, l2_weight=0.5)
        opt = LBFGS(tolerance=1e-12, max_iterations=6)
        opt.start(obj, dev, torch.zeros(dev.dim, dtype=torch.float64, device="cuda"))
        for _ in range(6):
            st = opt.step(obj, dev)
        torch.cuda.synchronize()
        out.append((st.coefficients.clone(), float(st.loss), st.gradient.clone()))
    (xa, fa, ga), (xb, fb, gb) = out
    assert torch.equal(xa, xb), float((xa - xb).abs().max())
    assert fa == fb
    assert torch.equal(ga, gb), float((ga - gb).abs().max())


@pytest.mark.parametrize("precision", ["f64", "bf16"])
def test_fused_offset_update_is_bitwise_set_offsets(precision):
    """``set_offsets_sum(base, part)`` (one pass: sum, cast, cached-margin shift) vs ``set_offsets(base + part)``:
    the same offsets, the same cached margins, and the same next value / gradient."""
    data, a = _dev_data(precision)
    _, b = _dev_data(precision)
    obj = GLMObjective(LOGISTIC, l2_weight=1.0)
    w = torch.from_numpy(np.random.default_rng(3).normal(size=a.dim) * 0.05).cuda()
    for x in (a, b):
        obj.calculate(x, w)                       # margins cached: the offset change shifts them
    g = torch.Generator(device="cuda").manual_seed(7)
    base = torch.randn(a.n_rows, generator=g, device="cuda", dtype=torch.float64) * 0.1
    part = torch.randn(a.n_rows, generator=g, device="cuda", dtype=torch.float64) * 0.1
    assert a.set_offsets_sum(base, part)
    b.set_offsets(base + part)
    assert torch.equal(a.o, b.o)
    za, zb = getattr(a, "z_cache", None), getattr(b, "z_cache", None)
    assert (za is None) == (zb is None)
    if za is not None:
        assert torch.equal(za[:a.n_rows], zb[:b.n_rows])
    fa, ga = obj.calculate(a, w)
    fb, gb = obj.calculate(b, w)
    assert float(fa) == float(fb) and torch.equal(ga, gb)


@pytest.mark.parametrize("precision", ["f64", "f32", "bf16"])
def test_perm_cast_is_bitwise_gather_then_cast(precision):
    """``_vec``'s one-launch gather + cast vs the torch expression ``w[perm].to(dtype)``."""
    from photon_ml_amd.ops.native import perm_cast
    _, dev = _dev_data(precision)
    w = torch.from_numpy(np.random.default_rng(4).normal(size=dev.dim) * 3.0).cuda()
    perm = dev.old_of_new
    ref = (w if perm is None else w[perm]).to(dev.vdt)
    assert torch.equal(dev._vec(w), ref)
    assert torch.equal(perm_cast(w, None, dev.vdt), w.to(dev.vdt))
    p = torch.randperm(w.numel(), device="cuda")
    assert torch.equal(perm_cast(w, p, dev.vdt), w[p].to(dev.vdt))


def _re_update(data, task, overlap, monkeypatch, resident="auto", hess=True):
    import photon_ml_amd.optimization.entity_tron as et
    if not hess:
        monkeypatch.setattr(et, "HESS_DMAX", 0)          # d_e 41: the sparse streaming kernels, not the tall one
    from photon_ml_amd.algorithm.coordinates import RandomEffectCoordinate
    from photon_ml_amd.data.random_effect import RandomEffectDataConfiguration
    from photon_ml_amd.optimization.config import (GLMOptimizationConfiguration, OptimizerConfig,
                                                   RegularizationContext)
    monkeypatch.setenv("PML_RE_OVERLAP", "1" if overlap else "0")
    monkeypatch.setattr(et, "RESIDENT", resident)
    cfg = GLMOptimizationConfiguration(OptimizerConfig("TRON", 30, 1e-10), RegularizationContext("L2"), 1.0)
    c = RandomEffectCoordinate("u", data, RandomEffectDataConfiguration("userId", "user"), cfg, task,
                               device="cuda", layout="segmented")
    m1 = c.update_model(c.initialize_model())
    s1 = c.score(m1)
    m2 = c.update_model(m1, partial_score=torch.from_numpy(np.sin(np.arange(data.n_rows)) * 0.2))
    torch.cuda.synchronize()
    return c, m1.values.copy(), s1.cpu(), m2.values.copy(), c.score(m2).cpu()


@pytest.mark.parametrize("task", ["LOGISTIC_REGRESSION", "POISSON_REGRESSION"])
def test_re_side_stream_overlap_is_bitwise_serial(task, monkeypatch):
    """The row-space solve on a side stream concurrent with the fused primal launch vs both serial: the two
    touch disjoint entities, so models and scores are bitwise equal."""
    data, _ = generate_game_data(n_rows=30000, n_users=700, d_user=40, seed=26, task=task)
    ra = _re_update(data, task, True, monkeypatch)
    rb = _re_update(data, task, False, monkeypatch)
    rs, fz, _ = ra[0]._comps
    assert rs is not None and fz is not None            # both components present: the overlap ran
    for i in range(1, 5):
        assert np.array_equal(np.asarray(ra[i]), np.asarray(rb[i])), i


def test_resident_error_check_runs_after_the_side_stream_launch(monkeypatch):
    """With register-resident tail tasks AND the overlap on, the fused solve returns its device error flag
    unread; the coordinate reads it only after the row-space solve was queued on the side stream."""
    import photon_ml_amd.optimization.entity_tron as et
    from photon_ml_amd.optimization.row_space import RowSpaceBatch
    events = []
    real_solve, real_check = RowSpaceBatch.solve, et.FusedResult.check_error

    def solve(self, *a, **k):
        events.append("rs_solve")
        return real_solve(self, *a, **k)

    def check(self):
        events.append("check_error" if self.err is not None else "check_none")
        return real_check(self)

    monkeypatch.setattr(RowSpaceBatch, "solve", solve)
    monkeypatch.setattr(et.FusedResult, "check_error", check)
    data, _ = generate_game_data(n_rows=60000, n_users=300, d_user=40, seed=28, task="LOGISTIC_REGRESSION")
    c = _re_update(data, "LOGISTIC_REGRESSION", True, monkeypatch, resident="force", hess=False)[0]
    fz = c._comps[1]
    assert fz.res is not None and fz.res["n"] > 0
    assert "check_error" in events
    first_check = events.index("check_error")
    assert "rs_solve" in events[:first_check], events


def test_device_csr_router_matches_scipy_router():
    """``RowRouter.forward_csr_device`` (entry permutation on the GPU, kept as a DeviceCSR) vs ``forward_csr``."""
    import scipy.sparse as sp
    from photon_ml_amd.parallel.sharding import RowRouter
    rng = np.random.default_rng(9)
    x = sp.random(5000, 800, density=0.02, format="csr", random_state=9, data_rvs=lambda k: rng.normal(size=k))
    x.sort_indices()
    r = RowRouter(torch.zeros(5000, dtype=torch.int64, device="cuda"))
    a = r.forward_csr(x)
    b = r.forward_csr_device(x, "cuda")
    assert torch.equal(b.indptr.cpu(), torch.from_numpy(a.indptr.astype(np.int64)))
    assert torch.equal(b.indices.cpu().to(torch.int64), torch.from_numpy(a.indices.astype(np.int64)))
    assert torch.equal(b.data.cpu(), torch.from_numpy(a.data.astype(np.float64)))


def test_heavy_tail_entities_take_the_pass_path_on_their_own_stream(monkeypatch):
    """Tail entities longer than one register-resident launch holds (here: RES_KMAX = 4 workgroups of 384 rows)
    leave the fused batch for the block-diagonal pass path, which runs on its own stream next to the fused launch:
    the same models and scores as the serial order (bitwise), and close to the all-streaming solve."""
    import photon_ml_amd.optimization.entity_tron as et
    monkeypatch.setattr(et, "RES_KMAX", 4)
    data, _ = generate_game_data(n_rows=60000, n_users=300, d_user=40, seed=28, task="LOGISTIC_REGRESSION")
    ra = _re_update(data, "LOGISTIC_REGRESSION", True, monkeypatch, hess=False)
    rs, fz, sub = ra[0]._comps
    assert fz is not None and fz.n_heavy > 0 and sub is not None and sub.entities.numel() >= fz.n_heavy
    rb = _re_update(data, "LOGISTIC_REGRESSION", False, monkeypatch, hess=False)
    for i in range(1, 5):
        assert np.array_equal(np.asarray(ra[i]), np.asarray(rb[i])), i
    rc = _re_update(data, "LOGISTIC_REGRESSION", True, monkeypatch, resident="0", hess=False)
    assert rc[0]._comps[1].n_heavy == 0
    for i in range(1, 5):
        torch.testing.assert_close(torch.as_tensor(ra[i]), torch.as_tensor(rc[i]), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("precision", ["f64", "bf16"])
def test_cached_margins_kernel_matches_torch(precision):
    """``DeviceGLMData.margins`` from the cached margins in one pass (``cached_margins_kernel``: fma(t, zd, z0) - o)
    vs the torch sequence clone / add_ / cast / sub_ (the same values to the single fma rounding)."""
    from photon_ml_amd.ops.native import cached_margins
    g = torch.Generator(device="cuda").manual_seed(3)
    n = 100_003
    z0 = torch.randn(n + 5, generator=g, device="cuda", dtype=torch.float64)
    zd = torch.randn(n + 5, generator=g, device="cuda", dtype=torch.float64)
    o = torch.randn(n, generator=g, device="cuda", dtype=torch.float64).to(
        torch.float64 if precision == "f64" else torch.float32)
    t = 0.37
    ref = (z0[:n] + t * zd[:n]) - o.to(torch.float64)
    out = cached_margins(z0, zd, t, o, n)
    assert out.shape == (n,)
    torch.testing.assert_close(out, ref, rtol=1e-15, atol=1e-15)
    assert torch.equal(cached_margins(z0, None, 0.0, None, n), z0[:n])
    assert torch.equal(cached_margins(z0, None, 0.0, o, n), z0[:n] - o.to(torch.float64))
    # through the data object: the scores of the last accepted point equal a fresh forward pass
    data, dev = _dev_data(precision)
    obj = GLMObjective(LOGISTIC, l2_weight=1.0)
    from photon_ml_amd.optimization.lbfgs import LBFGS
    opt = LBFGS(tolerance=1e-12, max_iterations=3)
    opt.start(obj, dev, torch.zeros(dev.dim, dtype=torch.float64, device="cuda"))
    for _ in range(3):
        st = opt.step(obj, dev)
    z_cached = dev.margins(st.coefficients)
    dev.z_cache = None                                   # force the forward pass
    z_fwd = dev.margins(st.coefficients)
    # (bf16 / fp32 shards: a pass gathers the coefficients cast to fp32, the cached margins come from the cast
    # direction; they agree to that rounding)
    tol = 1e-9 if precision == "f64" else 2e-6
    torch.testing.assert_close(z_cached, z_fwd, rtol=tol, atol=tol)
