"""Objective-function checks against central finite differences and GLM end-to-end quality gates.

Reference: ``photon-api/src/integTest/.../function/DistributedObjectiveFunctionTest.scala:406-586`` (gradient
and Hessian-vector vs finite differences, delta 1e-6, relative-or-absolute error < 1e-3, for every task x
{no reg, L2} x {benign, outlier-free weighted data} x normalization) and ``supervised/BaseGLMTest.scala:164-227``
(logistic L-BFGS on 10k x 10 synthetic: training AUC >= 0.95; linear: max |prediction - label| <= 1e-2).
"""
import numpy as np
import pytest
import torch

from photon_ml_amd.data.matrix import LabeledData
from photon_ml_amd.data.synthetic import generate_glm_data
from photon_ml_amd.diagnostics.evaluation import binary_metrics, AREA_UNDER_RECEIVER_OPERATOR_CHARACTERISTICS
from photon_ml_amd.estimators.game_estimator import train_generalized_linear_model
from photon_ml_amd.function.losses import loss_for_task
from photon_ml_amd.function.objective import GLMObjective
from photon_ml_amd.normalization.context import NormalizationContext, NormalizationType
from photon_ml_amd.ops.reference import TorchGLMData
from photon_ml_amd.optimization.config import RegularizationContext
from photon_ml_amd.stat.summary import BasicStatisticalSummary

DELTA = 1e-6
TOL = 1e-3
TASKS = ["LOGISTIC_REGRESSION", "POISSON_REGRESSION", "LINEAR_REGRESSION", "SMOOTHED_HINGE_LOSS_LINEAR_SVM"]


def _data(task, weighted, seed=3):
    ld, _ = generate_glm_data(task, 400, 12, density=0.4, seed=seed)
    if weighted:
        rng = np.random.default_rng(seed)
        ld = LabeledData(ld.x, ld.y, rng.normal(scale=0.1, size=ld.n_rows), rng.random(ld.n_rows) + 0.5)
    return ld


def _close(a, b):
    return abs(a - b) <= TOL * max(1.0, abs(a), abs(b))


@pytest.mark.parametrize("task", TASKS)
@pytest.mark.parametrize("l2", [0.0, 1.0])
@pytest.mark.parametrize("weighted", [False, True])
@pytest.mark.parametrize("norm", ["NONE", "STANDARDIZATION"])
def test_gradient_and_hessian_vs_finite_differences(task, l2, weighted, norm):
    ld = _data(task, weighted)
    nc = None
    if norm != "NONE":
        nc = NormalizationContext.build(NormalizationType.parse(norm), BasicStatisticalSummary.compute(ld.x),
                                        intercept_id=ld.n_features - 1)
    obj = GLMObjective(loss_for_task(task), l2, nc)
    data = TorchGLMData(ld)
    rng = np.random.default_rng(0)
    w = torch.from_numpy(rng.normal(scale=0.2, size=ld.n_features))
    f, g = obj.calculate(data, w)
    for j in range(ld.n_features):
        e = torch.zeros_like(w)
        e[j] = DELTA
        fd = (obj.value(data, w + e) - obj.value(data, w - e)) / (2 * DELTA)
        assert _close(float(g[j]), fd), (j, float(g[j]), fd)
    if obj.twice_differentiable:
        v = torch.from_numpy(rng.normal(size=ld.n_features))
        hv = obj.hessian_vector(data, w, v)
        fd_hv = (obj.gradient(data, w + DELTA * v) - obj.gradient(data, w - DELTA * v)) / (2 * DELTA)
        for j in range(ld.n_features):
            assert _close(float(hv[j]), float(fd_hv[j])), (j, float(hv[j]), float(fd_hv[j]))


def test_logistic_training_auc():
    """BaseGLMTest: logistic L-BFGS on 10k x 10 "numerically benign" binary data (SparkTestUtils: class-separable
    first attribute, x0 = +-(0.1 + 0.9u), remaining features sparse noise) reaches training AUC >= 0.95."""
    rng = np.random.default_rng(5)
    n, d = 10_000, 10
    y = (rng.random(n) <= 0.5).astype(np.float64)
    x0 = (0.1 + 0.9 * rng.random(n)) * np.where(y > 0, 1.0, -1.0)
    noise = rng.normal(size=(n, d - 2)) * (rng.random((n, d - 2)) < 0.1)
    import scipy.sparse as sp
    x = sp.csr_matrix(np.column_stack([x0, noise, np.ones(n)]))
    ld = LabeledData(x, y)
    m = train_generalized_linear_model(ld, "LOGISTIC_REGRESSION", "LBFGS", RegularizationContext("L2"), [0.1],
                                       max_iterations=100, tolerance=1e-7, device="cpu")[0][1]
    p = torch.sigmoid(torch.from_numpy(ld.x @ m.coefficients.means.numpy()))
    assert binary_metrics(p, ld.y)[AREA_UNDER_RECEIVER_OPERATOR_CHARACTERISTICS] >= 0.95
    assert bool(torch.isfinite(p).all())


def test_linear_regression_max_error():
    """BaseGLMTest: linear L-BFGS on 10k x 10 synthetic, noise sigma 1e-3 -> max |pred - label| <= 1e-2."""
    ld, _ = generate_glm_data("LINEAR_REGRESSION", 10_000, 10, density=0.9, seed=6, noise=1e-3)
    m = train_generalized_linear_model(ld, "LINEAR_REGRESSION", "LBFGS", RegularizationContext("NONE"), [0.0],
                                       max_iterations=200, tolerance=1e-12, device="cpu")[0][1]
    pred = ld.x @ m.coefficients.means.numpy()
    assert np.max(np.abs(pred - ld.y)) <= 1e-2


@pytest.mark.parametrize("task", TASKS)
@pytest.mark.parametrize("kind", ["benign", "outlier"])
@pytest.mark.parametrize("l2", [0.0, 1.0])
def test_finite_differences_on_reference_sample_families(task, kind, l2):
    """DistributedObjectiveFunctionTest.scala:406-437: gradient / Hessian-vector vs finite differences on the
    reference's benign AND outlier data families (SparkTestUtils generators, data/synthetic.draw_samples)."""
    from photon_ml_amd.data.synthetic import draw_samples
    ld = draw_samples(task, kind, seed=7, size=300, dimensionality=15)
    obj = GLMObjective(loss_for_task(task), l2)
    data = TorchGLMData(ld)
    rng = np.random.default_rng(1)
    w = torch.from_numpy(rng.normal(scale=0.2, size=ld.n_features))
    _, g = obj.calculate(data, w)
    for j in range(ld.n_features):
        e = torch.zeros_like(w)
        e[j] = DELTA
        fd = (obj.value(data, w + e) - obj.value(data, w - e)) / (2 * DELTA)
        assert _close(float(g[j]), fd), (j, float(g[j]), fd)
    if obj.twice_differentiable:
        v = torch.from_numpy(rng.normal(size=ld.n_features))
        hv = obj.hessian_vector(data, w, v)
        fd_hv = (obj.gradient(data, w + DELTA * v) - obj.gradient(data, w - DELTA * v)) / (2 * DELTA)
        for j in range(ld.n_features):
            assert _close(float(hv[j]), float(fd_hv[j])), (j, float(hv[j]), float(fd_hv[j]))
