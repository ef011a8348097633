"""Legacy per-model evaluation metrics (regression / binary classification / log-likelihood / AICc).

Reference: ``photon-diagnostics/.../Evaluation.scala:36-196``. Scores are the model MEAN function with offsets
(probability for logistic, exp for Poisson, the margin for linear / smoothed hinge). Metric names are the
reference's strings so reports and model selection keyed on them carry over:

* regression models (linear, Poisson): MAE, MSE, RMSE;
* binary classifiers (logistic, smoothed hinge): area under PR (Spark ``BinaryClassificationMetrics``: one point
  per distinct score threshold, curve starts at (recall 0, precision of the first threshold), trapezoids), area
  under ROC, peak F1 over thresholds;
* per-datum log-likelihood (logistic with scores clamped to [1e-9, 1-1e-9], Poisson with log Γ(y+1));
* AICc from the log-likelihood with the count of |w| > 1e-9 coefficients as the parameter count.

Everything is vectorised torch (CPU or GPU); the sort-based curves are O(n log n).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Callable, Dict, Optional

import numpy as np
import torch

from ..constants import TaskType
from ..models.glm import (GeneralizedLinearModel, LinearRegressionModel, LogisticRegressionModel,
                          PoissonRegressionModel, SmoothedHingeLossLinearSVMModel)

MEAN_ABSOLUTE_ERROR = "Mean absolute error"
MEAN_SQUARE_ERROR = "Mean square error"
ROOT_MEAN_SQUARE_ERROR = "Root mean square error"
AREA_UNDER_PRECISION_RECALL = "Area under precision/recall"
AREA_UNDER_RECEIVER_OPERATOR_CHARACTERISTICS = "Area under ROC"
PEAK_F1_SCORE = "Peak F1 score"
DATA_LOG_LIKELIHOOD = "Per-datum log likelihood"
AKAIKE_INFORMATION_CRITERION = "Akaike information criterion"
EPSILON = 1e-9

MetricsMap = Dict[str, float]


@dataclass(frozen=True)
class MetricMetadata:
    name: str
    description: str
    higher_is_better: bool
    value_range: Optional[tuple]


METRIC_METADATA = {m.name: m for m in [
    MetricMetadata(MEAN_ABSOLUTE_ERROR, "Regression metric", False, None),
    MetricMetadata(MEAN_SQUARE_ERROR, "Regression metric", False, None),
    MetricMetadata(ROOT_MEAN_SQUARE_ERROR, "Regression metric", False, None),
    MetricMetadata(AREA_UNDER_PRECISION_RECALL, "Binary classification metric", True, (0.0, 1.0)),
    MetricMetadata(AREA_UNDER_RECEIVER_OPERATOR_CHARACTERISTICS, "Binary classification metric", True, (0.0, 1.0)),
    MetricMetadata(DATA_LOG_LIKELIHOOD, "Model selection metric", True, None),
    MetricMetadata(AKAIKE_INFORMATION_CRITERION, "Model selection metric", False, None),
    MetricMetadata(PEAK_F1_SCORE, "Binary classification metric", True, (0.0, 1.0)),
]}


def _as_t(x, device=None):
    if isinstance(x, torch.Tensor):
        return x.to(device=device or x.device, dtype=torch.float64)
    return torch.as_tensor(np.asarray(x, dtype=np.float64), device=device)


def threshold_curve(scores: torch.Tensor, labels: torch.Tensor):
    """Cumulative (tp, fp) at each distinct score threshold, thresholds descending (Spark's binning-free curve)."""
    order = torch.argsort(scores, descending=True, stable=True)
    s = scores[order]
    pos = (labels[order] > 0.5).to(torch.float64)
    tp = torch.cumsum(pos, 0)
    fp = torch.cumsum(1.0 - pos, 0)
    last = torch.ones_like(s, dtype=torch.bool)
    if s.numel() > 1:
        last[:-1] = s[1:] != s[:-1]
    return s[last], tp[last], fp[last]


def binary_metrics(scores, labels) -> MetricsMap:
    s, tp, fp = threshold_curve(_as_t(scores), _as_t(labels))
    P = float(tp[-1]) if tp.numel() else 0.0
    N = float(fp[-1]) if fp.numel() else 0.0
    if P == 0 or N == 0:
        return {AREA_UNDER_PRECISION_RECALL: float("nan"), AREA_UNDER_RECEIVER_OPERATOR_CHARACTERISTICS: float("nan"),
                PEAK_F1_SCORE: float("nan")}
    recall = tp / P
    precision = tp / (tp + fp)
    fpr = fp / N
    zero = torch.zeros(1, dtype=torch.float64, device=tp.device)
    one = torch.ones(1, dtype=torch.float64, device=tp.device)
    # ROC: (0,0) + points + (1,1)
    rx = torch.cat([zero, fpr, one])
    ry = torch.cat([zero, recall, one])
    auroc = float(torch.trapezoid(ry, rx))
    # PR: (0, first precision) + points
    px = torch.cat([zero, recall])
    py = torch.cat([precision[:1], precision])
    aupr = float(torch.trapezoid(py, px))
    f1 = 2 * precision * recall / (precision + recall)
    return {AREA_UNDER_PRECISION_RECALL: aupr, AREA_UNDER_RECEIVER_OPERATOR_CHARACTERISTICS: auroc,
            PEAK_F1_SCORE: float(torch.nan_to_num(f1, nan=0.0).max())}


def regression_metrics(pred, labels) -> MetricsMap:
    d = _as_t(pred) - _as_t(labels)
    mse = float((d * d).mean())
    return {MEAN_ABSOLUTE_ERROR: float(d.abs().mean()), MEAN_SQUARE_ERROR: mse,
            ROOT_MEAN_SQUARE_ERROR: math.sqrt(mse)}


def logistic_log_likelihood(prob, labels) -> float:
    p = _as_t(prob)
    y = _as_t(labels)
    logp = torch.where(p > EPSILON, torch.log(p.clamp_min(EPSILON)), torch.full_like(p, math.log(EPSILON)))
    log1mp = torch.where(p > 1 - EPSILON, torch.full_like(p, math.log(EPSILON)), torch.log1p(-p.clamp(max=1 - EPSILON)))
    ll = y * logp + (1 - y) * log1mp
    if not bool(torch.isfinite(ll).all()):
        raise ValueError("non-finite logistic log-likelihood")
    return float(ll.mean())


def poisson_log_likelihood(margin, labels) -> float:
    z = _as_t(margin)
    y = _as_t(labels)
    return float((y * z - torch.exp(z) - torch.lgamma(1.0 + y)).mean())


def _predict(model: GeneralizedLinearModel, x, offsets, device):
    import scipy.sparse as sp
    w = model.coefficients.means.detach().cpu().numpy()
    margin = np.asarray(sp.csr_matrix(x) @ w).ravel()
    if offsets is not None:
        margin = margin + np.asarray(offsets)
    z = torch.from_numpy(margin).to(device)
    return z, model.mean_from_score(z)


def evaluate(model: GeneralizedLinearModel, data, device="cpu") -> MetricsMap:
    """Evaluation.evaluate(model, dataset) over a :class:`LabeledData`."""
    z, mean = _predict(model, data.x, data.offsets, device)
    y = torch.from_numpy(np.asarray(data.y, dtype=np.float64)).to(device)
    metrics: MetricsMap = {}
    if isinstance(model, (LinearRegressionModel, PoissonRegressionModel)):
        metrics.update(regression_metrics(mean, y))
    if isinstance(model, (LogisticRegressionModel, SmoothedHingeLossLinearSVMModel)):
        metrics.update(binary_metrics(mean, y))
    if isinstance(model, PoissonRegressionModel):
        metrics[DATA_LOG_LIKELIHOOD] = poisson_log_likelihood(z, y)
    elif isinstance(model, LogisticRegressionModel):
        metrics[DATA_LOG_LIKELIHOOD] = logistic_log_likelihood(mean, y)
    if DATA_LOG_LIKELIHOOD in metrics:
        n = len(y)
        ll = n * metrics[DATA_LOG_LIKELIHOOD]
        k = int((model.coefficients.means.abs() > 1e-9).sum())
        metrics[AKAIKE_INFORMATION_CRITERION] = 2.0 * (k - ll) + 2.0 * k * (k + 1) / (n - k - 1.0)
    return metrics


# ------------------------------------------------------------------------------------------------ model selection
def select_best_model(task, lambda_models, per_model_metrics: Dict[float, MetricsMap]):
    """ModelSelection.scala:26-91: linear -> min RMSE, Poisson -> max log-likelihood, classifiers -> max AUROC.

    Returns ``(lambda, model)``. Ties resolve to the first (largest λ) model.
    """
    task = TaskType.parse(task)
    if task == TaskType.LINEAR_REGRESSION:
        key, better = ROOT_MEAN_SQUARE_ERROR, (lambda a, b: a < b)
    elif task == TaskType.POISSON_REGRESSION:
        key, better = DATA_LOG_LIKELIHOOD, (lambda a, b: a > b)
    else:
        key, better = AREA_UNDER_RECEIVER_OPERATOR_CHARACTERISTICS, (lambda a, b: a > b)
    best = None
    for lam, model in lambda_models:
        v = per_model_metrics[lam][key]
        if best is None or better(v, best[2]):
            best = (lam, model, v)
    return best[0], best[1]
