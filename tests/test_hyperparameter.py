"""Hyper-parameter search + data validation tests.

Reference: ``photon-lib/src/test/.../hyperparameter/search/{RandomSearchTest,GaussianProcessSearchTest}.scala``
(Sobol candidates inside the ranges; GP search converges on a smooth objective), ``estimators/
GaussianProcessEstimatorTest.scala`` (GP interpolates noise-free data), ``criteria/ExpectedImprovementTest``
and ``photon-client/src/test/.../data/DataValidatorsTest.scala``.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from photon_ml_amd.data.validators import DataValidationError, sanity_check, validate
from photon_ml_amd.hyperparameter.search import (DoubleRange, ExpectedImprovement, GaussianProcessEstimator,
                                                 GaussianProcessSearch, Matern52, RandomSearch, EvaluationFunction)


class Quadratic(EvaluationFunction):
    higher_is_better = False

    def __init__(self, opt):
        self.opt = np.asarray(opt)
        self.calls = 0

    def __call__(self, c):
        self.calls += 1
        v = float(((np.asarray(c) - self.opt) ** 2).sum())
        return v, (np.asarray(c), v)

    def vectorize_params(self, o):
        return o[0]

    def get_evaluation_value(self, o):
        return o[1]


def test_double_range_parse():
    assert DoubleRange.parse("1e-4-1e4") == DoubleRange(1e-4, 1e4)
    assert DoubleRange.parse("-3-2") == DoubleRange(-3, 2)
    with pytest.raises(ValueError):
        DoubleRange(2, 1)


def test_random_search_in_range_and_prior_observations():
    fn = Quadratic([0.3, -1.0])
    rs = RandomSearch([DoubleRange(0, 1), DoubleRange(-2, 0)], fn)
    res = rs.find(16)
    pts = np.stack([r[0] for r in res])
    assert len(res) == 16 and fn.calls == 16
    assert (pts[:, 0] >= 0).all() and (pts[:, 0] <= 1).all() and (pts[:, 1] >= -2).all() and (pts[:, 1] <= 0).all()
    assert len(np.unique(pts, axis=0)) == 16
    prior = [fn(np.array([0.5, -0.5]))[1]]
    assert len(RandomSearch([DoubleRange(0, 1), DoubleRange(-2, 0)], fn).find(3, prior)) == 3


def test_gp_interpolates():
    x = np.linspace(0, 1, 8)[:, None]
    y = np.sin(4 * x[:, 0])
    model = GaussianProcessEstimator(Matern52(), True, burn_in=20, n_samples=10).fit(x, y)
    m, v = model.predict(x)
    assert np.allclose(m, y, atol=1e-3) and (v < 1e-3).all()


def test_expected_improvement_direction():
    ei = ExpectedImprovement(False, best=1.0)
    assert ei(np.array([0.5]), np.array([0.01]))[0] > ei(np.array([1.5]), np.array([0.01]))[0]


def test_gp_search_beats_random_on_smooth_objective():
    def run(cls):
        fn = Quadratic([0.7])
        kw = dict(burn_in=20, n_samples=10) if cls is GaussianProcessSearch else {}
        res = cls([DoubleRange(0, 1)], fn, **kw).find(10)
        return min(r[1] for r in res)
    assert run(GaussianProcessSearch) <= run(RandomSearch) + 1e-12
    assert run(GaussianProcessSearch) < 1e-3


def test_validators():
    x = sp.csr_matrix(np.array([[1.0, 0], [0, 2.0], [3.0, 1.0]]))
    y = np.array([0.0, 1.0, 1.0])
    assert validate("LOGISTIC_REGRESSION", y, np.zeros(3), np.ones(3), {"s": x}) == []
    msgs = validate("LOGISTIC_REGRESSION", np.array([0.0, 2.0, 1.0]), np.zeros(3), np.ones(3), {"s": x})
    assert any("non-binary" in m for m in msgs)
    assert validate("POISSON_REGRESSION", np.array([0.0, -1.0, 1.0]), None, None, {"s": x})
    bad = x.copy()
    bad.data[1] = np.inf
    assert validate("LINEAR_REGRESSION", y, None, None, {"s": bad})
    assert validate("LINEAR_REGRESSION", y, None, np.array([1.0, 0.0, 1.0]), {"s": x})
    assert validate("LINEAR_REGRESSION", y, np.array([0, np.nan, 0]), None, {"s": x})
    assert validate("LOGISTIC_REGRESSION", np.array([0.0, 2.0, 1.0]), None, None, {"s": x},
                    "VALIDATE_DISABLED") == []
    with pytest.raises(DataValidationError):
        sanity_check("LOGISTIC_REGRESSION", np.array([0.0, 2.0, 1.0]), None, None, {"s": x})


@pytest.mark.parametrize("task", ["LOGISTIC_REGRESSION", "POISSON_REGRESSION", "LINEAR_REGRESSION"])
def test_validators_on_reference_sample_families(task):
    """DataValidatorsTest: the reference's benign / outlier families pass FULL and SAMPLE validation; the
    invalid-feature and invalid-label families are rejected (SparkTestUtils.scala:85-308 generators)."""
    from photon_ml_amd.data.synthetic import draw_samples
    for kind in ("benign", "outlier"):
        ld = draw_samples(task, kind, seed=3, size=500, dimensionality=20)
        for mode in ("VALIDATE_FULL", "VALIDATE_SAMPLE"):
            assert validate(task, ld.y, ld.offsets, ld.weights, {"s": ld.x}, mode) == [], (kind, mode)
    bad_x = draw_samples(task, "invalid_features", seed=3, size=500, dimensionality=20)
    msgs = validate(task, bad_x.y, bad_x.offsets, bad_x.weights, {"s": bad_x.x})
    assert any("non-finite feature" in m for m in msgs)
    bad_y = draw_samples(task, "invalid_labels", seed=3, size=500, dimensionality=20)
    msgs = validate(task, bad_y.y, bad_y.offsets, bad_y.weights, {"s": bad_y.x})
    assert any("non-finite label" in m for m in msgs)
    with pytest.raises(DataValidationError):
        sanity_check(task, bad_y.y, None, None, {"s": bad_y.x})
    # scoring data may carry any label, but never non-finite features
    assert validate(task, bad_y.y, None, None, {"s": bad_y.x}, for_training=False) == []
    assert validate(task, bad_x.y, None, None, {"s": bad_x.x}, for_training=False)
