"""Optimizer tests mirroring photon-lib/src/test/.../optimization/{OptimizerTest,LBFGSTest,OWLQNTest,
OptimizationUtilsTest}.scala and the scikit-learn coefficient checks of
photon-api/src/integTest/.../estimators/GameEstimatorIntegTest.scala:79-178."""
import numpy as np
import pytest
import torch

from photon_ml_amd.data.matrix import LabeledData
from photon_ml_amd.function.losses import SQUARED, LOGISTIC
from photon_ml_amd.function.objective import GLMObjective
from photon_ml_amd.ops.reference import TorchGLMData
from photon_ml_amd.optimization import (LBFGS, OWLQN, TRON, ConvergenceReason, project_box)


class QuadraticData:
    """sum_j (w_j - c)^2 expressed through the GLMComputable interface (TestObjective.scala)."""

    def __init__(self, dim, centroid=4.0):
        self.dim = dim
        self.c = centroid
        self.n_rows = 1

    def value_grad_sums(self, loss, w_eff, shift):
        d = w_eff - self.c
        return float(torch.dot(d, d)), 0.0, 2.0 * d

    def hv_sums(self, loss, w_eff, shift, v_eff, vshift):
        return 2.0 * v_eff, 0.0


TRIVIAL = [
    (0.0, [-0.7306653538519616, 0.0]),
    (1.0, [0.6750417712898752, -0.4232874171873786]),
    (1.0, [0.1863463229359709, -0.8163423997075965]),
    (0.0, [-0.6719842051493347, 0.0]),
    (1.0, [0.9699938346531928, 0.0]),
    (1.0, [0.22759406190283604, 0.0]),
    (1.0, [0.9688721028330911, 0.0]),
    (0.0, [0.5993795346650845, 0.0]),
    (0.0, [0.9219423508390701, -0.8972778242305388]),
    (0.0, [0.7006904841584055, -0.5607635619919824]),
]


def trivial_data():
    y = np.array([t[0] for t in TRIVIAL])
    x = np.array([t[1] + [1.0] for t in TRIVIAL])
    return LabeledData(x, y)


@pytest.mark.parametrize("opt_cls", [LBFGS, TRON])
def test_converges_to_centroid(opt_cls):
    data = QuadraticData(5)
    obj = GLMObjective(SQUARED)
    opt = opt_cls(tolerance=1e-9, max_iterations=100)
    w, f = opt.optimize(obj, data, torch.zeros(5, dtype=torch.float64))
    assert torch.allclose(w, torch.full((5,), 4.0, dtype=torch.float64), atol=1e-4)
    assert f < 1e-6
    # objective monotone non-increasing across tracked states
    losses = [s.loss for s in opt.tracker.states]
    assert all(b <= a + 1e-12 for a, b in zip(losses, losses[1:]))
    assert opt.tracker.convergence_reason is not None


@pytest.mark.parametrize("lam,w_exp,f_exp", [(1.0, 3.5, 7.5), (2.0, 3.0, 14.0), (8.0, 0.0, 32.0)])
def test_owlqn_analytic(lam, w_exp, f_exp):
    """OWLQNTest.scala:45-47: minimise sum (w-4)^2 + lam ||w||_1 in 2-D."""
    data = QuadraticData(2)
    opt = OWLQN(lam, tolerance=1e-12, max_iterations=100)
    w, f = opt.optimize(GLMObjective(SQUARED), data, torch.zeros(2, dtype=torch.float64))
    assert np.allclose(w.numpy(), w_exp, atol=1e-6)
    assert abs(f - f_exp) < 1e-6


def test_box_constraints():
    data = QuadraticData(3)
    cons = {0: (-1.0, 1.0), 2: (4.5, 10.0)}
    for cls in (LBFGS, TRON):
        opt = cls(tolerance=1e-9, max_iterations=50, constraints=cons)
        w, _ = opt.optimize(GLMObjective(SQUARED), data, torch.zeros(3, dtype=torch.float64))
        assert w[0] <= 1.0 + 1e-12 and w[0] >= -1.0
        assert w[2] >= 4.5
    p = project_box(torch.tensor([-5.0, 0.5, 5.0], dtype=torch.float64), {0: (-1, 1), 2: (0, 2)})
    assert p.tolist() == [-1.0, 0.5, 2.0]


def test_linear_regression_matches_sklearn():
    """GameEstimatorIntegTest.simpleHardcodedTest: L2 lambda=0.3, LBFGS tol 1e-11 -> sklearn coefficients."""
    data = TorchGLMData(trivial_data())
    obj = GLMObjective(SQUARED, l2_weight=0.3)
    opt = LBFGS(tolerance=1e-11, max_iterations=100)
    w, _ = opt.optimize(obj, data, torch.zeros(3, dtype=torch.float64))
    expected = [0.3215554473500486, 0.17904355431985355, 0.4122241763914806]
    assert np.allclose(w.numpy(), expected, atol=1e-12, rtol=0)


def test_tron_matches_lbfgs_logistic():
    rng = np.random.default_rng(0)
    x = rng.normal(size=(500, 8))
    x[:, -1] = 1.0
    w_true = rng.normal(size=8)
    y = (rng.random(500) < 1 / (1 + np.exp(-x @ w_true))).astype(float)
    data = TorchGLMData(LabeledData(x, y))
    obj = GLMObjective(LOGISTIC, l2_weight=1.0)
    w1, f1 = LBFGS(tolerance=1e-10, max_iterations=200).optimize(obj, data, torch.zeros(8, dtype=torch.float64))
    w2, f2 = TRON(tolerance=1e-10, max_iterations=50).optimize(obj, data, torch.zeros(8, dtype=torch.float64))
    assert abs(f1 - f2) < 1e-7
    assert np.allclose(w1.numpy(), w2.numpy(), atol=1e-5)


@pytest.mark.parametrize("norm", [None, "STANDARDIZATION"])
@pytest.mark.parametrize("task", ["LOGISTIC_REGRESSION", "POISSON_REGRESSION", "LINEAR_REGRESSION"])
def test_margin_space_line_search_matches_full_evaluations(task, norm, monkeypatch):
    """L-BFGS with trial steps evaluated from cached margins (z0 + t zd; full gradient only at the accepted step)
    follows the same iterates as the line search that evaluates the full objective at every trial."""
    import photon_ml_amd.optimization.lbfgs as lb
    from photon_ml_amd.data.synthetic import generate_glm_data
    from photon_ml_amd.function.losses import loss_for_task
    from photon_ml_amd.function.objective import GLMObjective
    from photon_ml_amd.normalization.context import NormalizationContext
    from photon_ml_amd.ops.reference import TorchGLMData
    from photon_ml_amd.stat.summary import BasicStatisticalSummary
    data, _ = generate_glm_data(task, 2000, 25, density=0.3, seed=4)
    nc = NormalizationContext.build(norm, BasicStatisticalSummary.compute(data.x), data.n_features - 1) if norm \
        else None
    gd = TorchGLMData(data, "cpu")
    out = {}
    for mode in (False, True):
        monkeypatch.setattr(lb, "MARGIN_LINE_SEARCH", mode)
        obj = GLMObjective(loss_for_task(task), 0.5, nc)
        opt = lb.LBFGS(tolerance=1e-12, max_iterations=25)
        w, f = opt.optimize(obj, gd, torch.zeros(25, dtype=torch.float64))
        out[mode] = (w, f, obj.n_value_grad, opt.current.iter)
    (w0, f0, n0, i0), (w1, f1, n1, i1) = out[False], out[True]
    assert i0 == i1
    assert torch.allclose(w0, w1, rtol=1e-8, atol=1e-10) and abs(f0 - f1) <= 1e-10 * abs(f0)
    assert n1 <= n0  # full (forward + transpose) evaluations: only initial state + one per accepted step


@pytest.mark.parametrize("norm", [None, "STANDARDIZATION"])
@pytest.mark.parametrize("task", ["LOGISTIC_REGRESSION", "POISSON_REGRESSION", "LINEAR_REGRESSION"])
def test_tron_margin_space_trial_matches_full_evaluations(task, norm):
    """TRON with each trial point w + s evaluated from margins accumulated during CG (z(w) + sum alpha_i X d_i,
    normalization shifts included) follows the same iterates as evaluating the full objective at w + s."""
    from photon_ml_amd.data.synthetic import generate_glm_data
    from photon_ml_amd.function.losses import loss_for_task
    from photon_ml_amd.normalization.context import NormalizationContext
    from photon_ml_amd.stat.summary import BasicStatisticalSummary
    data, _ = generate_glm_data(task, 2000, 25, density=0.3, seed=5)
    nc = NormalizationContext.build(norm, BasicStatisticalSummary.compute(data.x), data.n_features - 1) if norm \
        else None
    gd = TorchGLMData(data, "cpu")
    out = {}
    for mode in (False, True):
        obj = GLMObjective(loss_for_task(task), 0.5, nc)
        opt = TRON(tolerance=1e-12, max_iterations=15)
        opt.margin_trial = mode
        w, f = opt.optimize(obj, gd, torch.zeros(25, dtype=torch.float64))
        out[mode] = (w, f, opt.current.iter, opt.total_cg_iterations)
    (w0, f0, i0, c0), (w1, f1, i1, c1) = out[False], out[True]
    assert (i0, c0) == (i1, c1)
    assert torch.allclose(w0, w1, rtol=1e-8, atol=1e-10) and abs(f0 - f1) <= 1e-10 * abs(f0)


def test_vector_free_two_loop_matches_recursion():
    """The Gram-matrix (vector-free) two-loop used for long device vectors and feature shards == the classic
    two-loop recursion."""
    from photon_ml_amd.optimization.lbfgs import _History
    rng = np.random.default_rng(3)
    h = _History(5)
    A = rng.normal(size=(40, 40))
    A = A @ A.T + 40 * np.eye(40)
    for _ in range(7):
        s = torch.from_numpy(rng.normal(size=40))
        h.push(s, torch.from_numpy(A) @ s)
    g = torch.from_numpy(rng.normal(size=40))
    torch.testing.assert_close(h._apply_inverse_gram(g), h.apply_inverse(g), rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("norm", [None, "STANDARDIZATION"])
@pytest.mark.parametrize("opt_name,tol", [("LBFGS", 1e-3), ("LBFGS", 1e-12), ("TRON", 1e-4)])
def test_lazy_zero_point_gradient_tolerance(opt_name, tol, norm, monkeypatch):
    """The zero point's gradient norm (tolerance scale, Optimizer.scala / Appendix C.7) as an upper bound from
    one elementwise pass, made exact only when a gradient norm comes within the bound: the same iterates, stop
    reasons and tolerances as the eager zero-point evaluation, and no zero-point gradient pass at all while the
    gradient stays above the bound (tolerance 1e-12)."""
    import photon_ml_amd.optimization.optimizer as om
    from photon_ml_amd.data.synthetic import generate_glm_data
    from photon_ml_amd.normalization.context import NormalizationContext
    from photon_ml_amd.stat.summary import BasicStatisticalSummary
    data, _ = generate_glm_data("LOGISTIC_REGRESSION", 3000, 20, density=0.3, seed=5)
    nc = NormalizationContext.build(norm, BasicStatisticalSummary.compute(data.x), data.n_features - 1) if norm \
        else None
    gd = TorchGLMData(data, "cpu")
    calls = []
    orig = GLMObjective.calculate

    def spy(self, d, w):
        calls.append(bool(getattr(w, "_pml_zero", False)))
        return orig(self, d, w)

    monkeypatch.setattr(GLMObjective, "calculate", spy)
    out = {}
    for lazy in (False, True):
        monkeypatch.setattr(om, "LAZY_ZERO_GRADIENT", lazy)
        calls.clear()
        obj = GLMObjective(LOGISTIC, 0.5, nc)
        opt = (LBFGS if opt_name == "LBFGS" else TRON)(tolerance=tol, max_iterations=40)
        w, f = opt.optimize(obj, gd, torch.full((20,), 0.01, dtype=torch.float64))
        opt._resolve_grad_tol()
        out[lazy] = (w, f, opt.current.iter, opt.convergence_reason(), opt.loss_abs_tol, opt.grad_abs_tol,
                     sum(calls))
    a, b = out[False], out[True]
    assert torch.equal(a[0], b[0]) and a[1] == b[1] and a[2] == b[2] and a[3] == b[3]
    assert a[4] == b[4] and abs(a[5] - b[5]) <= 1e-12 * abs(a[5])
    assert a[6] == 1                         # eager: the zero point's full evaluation
    if tol == 1e-12:
        assert b[6] == 1 and a[3] != ConvergenceReason.GRADIENT_CONVERGED   # only the final resolve above
