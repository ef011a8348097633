"""Whole-iteration L-BFGS plans (``optimization/lbfgs.py`` PLAN): the next iteration's direction, margin pass,
gradient at t = 1 and history pair are queued before the current step is validated, into the other buffer pair of
the double-buffered margin cache (``DeviceGLMData.ls_begin(alt=True)``), and read back in one synchronisation.

The planned run must reproduce the unplanned one BITWISE (same decisions on the same values), leave the data's
margin cache at the last accepted point when the optimizer stops with a plan outstanding, and fall back correctly
when a plan is rejected (forced here every few plans: the fallback recomputes the first trial's gradient input,
whose rounding may differ in the last bit from the direction pass's, so that case is compared at 1e-10)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _problem(seed=21, precision="f64"):
    from photon_ml_amd.data.synthetic import generate_device_shard
    data, w = generate_device_shard(200_000, 40_000, 20, "cuda", precision, seed=seed, chunk_rows=1 << 16,
                                    layout="tiled")
    data.set_offsets(0.05 * torch.randn(data.n_rows, dtype=torch.float64, device="cuda",
                                        generator=torch.Generator(device="cuda").manual_seed(seed)))
    return data


def _fit(monkeypatch, plan, reject=0, precision="f64", tol=1e-12, iters=20, warm=None, seed=21):
    import photon_ml_amd.optimization.lbfgs as lb
    from photon_ml_amd.function.losses import LOGISTIC
    from photon_ml_amd.function.objective import GLMObjective
    monkeypatch.setattr(lb, "PLAN", plan)
    monkeypatch.setattr(lb, "PLAN_TEST_REJECT", reject)
    data = _problem(seed, precision)
    obj = GLMObjective(LOGISTIC, 0.5)
    opt = lb.LBFGS(tolerance=tol, max_iterations=iters)
    w0 = torch.zeros(data.dim, dtype=torch.float64, device="cuda")
    w, f = opt.optimize(obj, data, w0)
    res = [(w, f, opt.current.iter, opt.plans_used, opt.wasted_spec_passes)]
    if warm:
        # GAME-style: new offsets, warm start from the last model on the same data object
        data.set_offsets(0.03 * torch.randn(data.n_rows, dtype=torch.float64, device="cuda",
                                            generator=torch.Generator(device="cuda").manual_seed(5)))
        w, f = opt.optimize(obj, data, w)
        res.append((w, f, opt.current.iter, opt.plans_used, opt.wasted_spec_passes))
    return res, data, obj


@pytest.mark.parametrize("precision", ["f64", "bf16"])
def test_planned_lbfgs_is_bitwise_the_unplanned_one(precision, monkeypatch):
    ref, _, _ = _fit(monkeypatch, False, precision=precision, warm=True)
    got, _, _ = _fit(monkeypatch, True, precision=precision, warm=True)
    for (w0, f0, i0, _, _), (w1, f1, i1, used, _) in zip(ref, got):
        assert i0 == i1 and f0 == f1 and torch.equal(w0, w1)
    assert got[-1][3] > 0, "no iteration ran from a plan"


def test_plan_outstanding_at_convergence_leaves_cache_at_accepted_point(monkeypatch):
    """Stopping on the loss tolerance with a plan queued: the speculative passes are abandoned and the cached
    margins (used for scoring) are those of the returned coefficients."""
    import photon_ml_amd.optimization.lbfgs as lb
    monkeypatch.setattr(lb, "SPECULATE_LOSS_MARGIN", 0.0)     # always plan ahead, also next to the tolerance
    (res,), data, _ = _fit(monkeypatch, True, tol=1e-4, iters=400)
    w = res[0]
    assert res[2] < 400 and res[4] >= 1          # stopped on the tolerance with a plan queued
    cached = data.margins(w)
    fresh = _problem().margins(w)            # the same shard rebuilt: no cache, a forward pass
    assert torch.allclose(cached, fresh, rtol=1e-10, atol=1e-10)


def test_rejected_plans_fall_back_to_the_search(monkeypatch):
    ref, _, _ = _fit(monkeypatch, False, warm=True)
    got, _, _ = _fit(monkeypatch, True, reject=2, warm=True)
    for (w0, f0, i0, _, _), (w1, f1, i1, _, _) in zip(ref, got):
        assert i0 == i1
        assert abs(f0 - f1) <= 1e-12 * abs(f0)
        assert torch.allclose(w0, w1, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("precision", ["f64", "bf16"])
def test_ls_eval_many_is_bitwise_the_single_trials(precision):
    """ls_eval_multi_kernel: (F, D) at each step of a ladder in one pass == ls_eval at that step alone, bitwise."""
    from photon_ml_amd.function.losses import LOGISTIC
    from photon_ml_amd.function.objective import GLMObjective
    data = _problem(7, precision)
    obj = GLMObjective(LOGISTIC, 0.5)
    w = torch.zeros(data.dim, dtype=torch.float64, device="cuda")
    f, g = obj.calculate(data, w)
    d = -g
    mls = obj.margin_line_search(data, w, d, 1e-3)
    assert mls is not None
    ts = [2e-3 * 1.5 ** k for k in range(6)]
    many = data.ls_eval_many(LOGISTIC, ts)
    for t, (F, D) in zip(ts, many):
        F1, D1 = data.ls_eval(LOGISTIC, t)
        assert (F, D) == (F1, D1), (t, F, F1, D, D1)
    for k in (1, 3):
        assert data.ls_eval_many(LOGISTIC, ts[:k]) == many[:k]


def _fit_gated(monkeypatch, gated, disagree=False, precision="f64"):
    import photon_ml_amd.optimization.lbfgs as lb
    monkeypatch.setattr(lb, "GATED_FINISH", gated)
    monkeypatch.setattr(lb, "GATED_TEST_DISAGREE", disagree)
    return _fit(monkeypatch, False, precision=precision, warm=True)


@pytest.mark.parametrize("precision", ["f64", "bf16"])
def test_gated_first_trial_finish_is_bitwise_the_host_path(precision, monkeypatch):
    """The device-decided, gated gradient pass at t = 1 (ls_gate_kernel + gated tl_t_multi) gives bitwise the
    iterates of the host-decided finish; when the host does not keep the gated results (forced here), restoring the
    line-search state and searching again matches to rounding (the first trial's gradient input is recomputed)."""
    ref, _, _ = _fit_gated(monkeypatch, False, precision=precision)
    got, data, _ = _fit_gated(monkeypatch, True, precision=precision)
    for (w0, f0, i0, _, _), (w1, f1, i1, _, _) in zip(ref, got):
        assert i0 == i1 and f0 == f1 and torch.equal(w0, w1)
    dis, _, _ = _fit_gated(monkeypatch, True, disagree=True, precision=precision)
    for (w0, f0, i0, _, _), (w1, f1, i1, _, _) in zip(ref, dis):
        assert i0 == i1 and abs(f0 - f1) <= 1e-12 * abs(f0) and torch.allclose(w0, w1, rtol=1e-9, atol=1e-12)


def test_gated_transpose_does_no_work_when_the_gate_is_closed():
    """pml_set_gate with a 0 flag: the shard-wide transpose leaves its output untouched; with 1 it is the plain
    pass."""
    from photon_ml_amd.function.losses import LOGISTIC
    data = _problem(9)
    c = torch.randn(data.n_rows, dtype=torch.float64, device="cuda").to(data.coef.dtype)
    G_ref = torch.zeros(data.dim, dtype=torch.float64, device="cuda")
    data.t_all(c, G_ref)
    gate = torch.zeros(1, dtype=torch.int32, device="cuda")
    for flag in (0, 1):
        gate.fill_(flag)
        G = torch.full((data.dim,), 7.0, dtype=torch.float64, device="cuda")
        if flag:
            G.zero_()
        data.parts.zero_()          # (split tiles are combined from this scratch even when no item ran)
        data.lib.pml_set_gate(gate.data_ptr())
        try:
            data.t_all(c, G)
        finally:
            data.lib.pml_set_gate(None)
        torch.cuda.synchronize()
        if flag:
            assert torch.equal(G, G_ref)
        else:
            assert bool((G == 7.0).all())       # no item ran; the split-tile combine added zeros
