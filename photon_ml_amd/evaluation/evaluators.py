"""Evaluators over score arrays aligned with the samples (no joins: scores, labels, offsets, weights and group ids
share the sample order).

Reference: ``photon-lib/.../evaluation/{Evaluator,EvaluatorType}.scala`` (evaluate = f(score + offset), betterThan),
``photon-api/.../evaluation/*.scala``:
  * AUC (global; MLlib BinaryClassificationMetrics -> UNWEIGHTED, Appendix C.5) ``AreaUnderROCCurveEvaluator``
  * local weighted AUC with tie groups ``AreaUnderROCCurveLocalEvaluator.scala:33-70``
  * RMSE = sqrt(sum w (z-y)^2/2 / N) — the reference's definition, kept for parity (Appendix C.1)
  * logistic / poisson / squared / smoothed-hinge loss sums
  * multi-evaluators grouped by an id tag: AUC:tag and PRECISION@k:tag, mean over groups with finite values
    (``MultiEvaluator.scala:49-64``, ``PrecisionAtKLocalEvaluator.scala:39-51``)
  * name parsing ``AUC``, ``RMSE``, ``LOGISTIC_LOSS``, ..., ``PRECISION@5:queryId``, ``AUC:userId``.

Sorting-based metrics run on the device (torch sort / segmented reductions), so the whole validation pass stays
in HBM.
"""
from __future__ import annotations

import math
import re
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from ..constants import POSITIVE_RESPONSE_THRESHOLD, TaskType
from ..function import losses as L


def _t(x, device=None):
    return torch.as_tensor(x, dtype=torch.float64, device=device)


def auc_weighted(scores: torch.Tensor, labels: torch.Tensor, weights: Optional[torch.Tensor] = None) -> float:
    """Weighted ROC AUC with tied scores counted as half (trapezoid), vectorised (K11)."""
    s = _t(scores)
    y = _t(labels, s.device)
    w = torch.ones_like(s) if weights is None else _t(weights, s.device)
    if s.numel() == 0:
        return float("nan")
    order = torch.argsort(s, descending=True, stable=True)
    s, y, w = s[order], y[order], w[order]
    pos = torch.where(y > POSITIVE_RESPONSE_THRESHOLD, w, torch.zeros_like(w))
    neg = w - pos
    # group ties
    new_group = torch.ones_like(s, dtype=torch.bool)
    new_group[1:] = s[1:] != s[:-1]
    gid = torch.cumsum(new_group.to(torch.int64), 0) - 1
    ng = int(gid[-1].item()) + 1
    gp = torch.zeros(ng, dtype=torch.float64, device=s.device).index_add_(0, gid, pos)
    gn = torch.zeros(ng, dtype=torch.float64, device=s.device).index_add_(0, gid, neg)
    tp_before = torch.cumsum(gp, 0) - gp
    raw = torch.sum(tp_before * gn + gp * gn / 2.0)
    tp, tn = gp.sum(), gn.sum()
    return float(raw / (tp * tn))


def precision_at_k(scores, labels, k: int) -> float:
    s = _t(scores)
    y = _t(labels, s.device)
    order = torch.argsort(s, descending=True, stable=True)[:k]
    hits = int((y[order] > POSITIVE_RESPONSE_THRESHOLD).sum())
    return hits / k


def _dist():
    from ..parallel.dist import is_dist
    return is_dist()


def _allsum(*vals: float) -> List[float]:
    """Sum scalars over the process group (one collective)."""
    from ..parallel.dist import all_reduce_
    from ..parallel.sharding import comm_device
    t = torch.tensor(vals, dtype=torch.float64, device=comm_device())
    all_reduce_(t)
    return t.tolist()


def _gather(t: torch.Tensor) -> torch.Tensor:
    from ..parallel.sharding import all_gather_varlen
    return torch.cat([x.to(t.device) for x in all_gather_varlen(t.detach().cpu())])


class Evaluator:
    """Evaluates ``scores + offsets`` against the labels. Under a process group every rank holds a row shard:
    additive metrics (losses, RMSE) all-reduce their sums, rank metrics (AUC, per-group metrics) all-gather the
    (score, label[, weight, group]) columns first."""

    name = "EVALUATOR"
    higher_is_better = True

    def __init__(self, labels, offsets=None, weights=None, device=None):
        self.distributed = _dist()
        self.labels = _t(labels, device)
        n = self.labels.numel()
        self.offsets = torch.zeros(n, dtype=torch.float64, device=self.labels.device) if offsets is None else _t(
            offsets, self.labels.device)
        self.weights = torch.ones(n, dtype=torch.float64, device=self.labels.device) if weights is None else _t(
            weights, self.labels.device)

    def evaluate(self, scores) -> float:
        s = _t(scores, self.labels.device) + self.offsets
        return self._evaluate(s)

    def _evaluate(self, s: torch.Tensor) -> float:
        raise NotImplementedError

    def better_than(self, a: float, b: float) -> bool:
        return a > b if self.higher_is_better else a < b

    def __repr__(self):
        return self.name


class AUCEvaluator(Evaluator):
    name = "AUC"

    def _evaluate(self, s):
        if self.distributed:
            return auc_weighted(_gather(s), _gather(self.labels), None)
        return auc_weighted(s, self.labels, None)  # MLlib AUC ignores weights


class RMSEEvaluator(Evaluator):
    name = "RMSE"
    higher_is_better = False

    def _evaluate(self, s):
        d = s - self.labels
        num, cnt = float(torch.sum(self.weights * 0.5 * d * d)), float(self.labels.numel())
        if self.distributed:
            num, cnt = _allsum(num, cnt)
        return math.sqrt(num / max(cnt, 1.0))


class _LossEvaluator(Evaluator):
    higher_is_better = False
    loss = None

    def evaluate(self, scores) -> float:
        s = _t(scores, self.labels.device)
        if s.is_cuda and s.dtype == torch.float64:
            # scores + offsets folded into the fused loss pass (no separate N-length add)
            from ..ops.native import loss_sum
            t = loss_sum(self.loss.loss_id, s.contiguous(), self.labels, self.weights, offsets=self.offsets)
            if t is not None:
                v = float(t)
                return _allsum(v)[0] if self.distributed else v
        return self._evaluate(s + self.offsets)

    def _evaluate(self, s):
        v = None
        if s.is_cuda:
            from ..ops.native import loss_sum
            t = loss_sum(self.loss.loss_id, s.contiguous(), self.labels, self.weights)   # one fused HIP pass
            v = None if t is None else float(t)
        if v is None:
            l, _ = self.loss.loss_and_dz(s, self.labels)
            v = float(torch.sum(self.weights * l))
        return _allsum(v)[0] if self.distributed else v


class LogisticLossEvaluator(_LossEvaluator):
    name = "LOGISTIC_LOSS"
    loss = L.LOGISTIC


class PoissonLossEvaluator(_LossEvaluator):
    name = "POISSON_LOSS"
    loss = L.POISSON


class SquaredLossEvaluator(_LossEvaluator):
    name = "SQUARED_LOSS"
    loss = L.SQUARED


class SmoothedHingeLossEvaluator(_LossEvaluator):
    name = "SMOOTHED_HINGE_LOSS"
    loss = L.SMOOTHED_HINGE


class MultiEvaluator(Evaluator):
    """Per-group local metric, mean over groups whose value is finite."""

    def __init__(self, ids, labels, offsets=None, weights=None, device=None):
        super().__init__(labels, offsets, weights, device)
        ids = np.asarray(ids)
        if self.distributed:  # groups can span ranks: gather group keys once, evaluate on the gathered columns
            from ..parallel.sharding import stable_hash64
            keys = _gather(torch.from_numpy(stable_hash64(ids))).numpy()
            uniq, inv = np.unique(keys, return_inverse=True)
            self.labels_all = _gather(self.labels)
            self.weights_all = _gather(self.weights)
        else:
            uniq, inv = np.unique(ids.astype(str) if ids.dtype == object else ids, return_inverse=True)
        self.group = torch.as_tensor(inv, dtype=torch.int64, device=self.labels.device)
        self.n_groups = len(uniq)

    def _local(self, s, y, w) -> float:
        raise NotImplementedError

    def _evaluate(self, s):
        order = torch.argsort(self.group, stable=True)
        g = self.group[order]
        if self.distributed:
            s, y, w = _gather(s)[order], self.labels_all[order], self.weights_all[order]
        else:
            s, y, w = s[order], self.labels[order], self.weights[order]
        counts = torch.bincount(g, minlength=self.n_groups).cpu().numpy()
        starts = np.concatenate([[0], np.cumsum(counts)])
        vals = []
        s_c, y_c, w_c = s.cpu(), y.cpu(), w.cpu()
        for i in range(self.n_groups):
            a, b = starts[i], starts[i + 1]
            if b > a:
                v = self._local(s_c[a:b], y_c[a:b], w_c[a:b])
                if math.isfinite(v):
                    vals.append(v)
        return float(np.mean(vals)) if vals else float("nan")


class AUCMultiEvaluator(MultiEvaluator):
    def __init__(self, id_tag: str, ids, labels, offsets=None, weights=None, device=None):
        super().__init__(ids, labels, offsets, weights, device)
        self.id_tag = id_tag
        self.name = f"AUC:{id_tag}"

    def _local(self, s, y, w):
        return auc_weighted(s, y, w)


class PrecisionAtKMultiEvaluator(MultiEvaluator):
    def __init__(self, k: int, id_tag: str, ids, labels, offsets=None, weights=None, device=None):
        if k <= 0:
            raise ValueError(f"Position k must be greater than 0: {k}")
        super().__init__(ids, labels, offsets, weights, device)
        self.k = k
        self.id_tag = id_tag
        self.name = f"PRECISION@{k}:{id_tag}"

    def _local(self, s, y, w):
        return precision_at_k(s, y, self.k)


# --------------------------------------------------------------------------------------------------------------
@dataclass(frozen=True)
class EvaluatorType:
    name: str
    id_tag: Optional[str] = None
    k: Optional[int] = None

    @property
    def is_multi(self) -> bool:
        return self.id_tag is not None

    def __str__(self):
        return self.name


SIMPLE_TYPES = ("AUC", "RMSE", "LOGISTIC_LOSS", "POISSON_LOSS", "SMOOTHED_HINGE_LOSS", "SQUARED_LOSS")
_P_AT_K = re.compile(r"(?i:PRECISION)@(\d+):(.*)")
_AUC_TAG = re.compile(r"(?i:AUC):(.*)")


def parse_evaluator_type(name: str) -> EvaluatorType:
    """``Utils.evaluatorParser`` (CLI/util/Utils.scala:308-322)."""
    n = name.strip()
    m = _P_AT_K.fullmatch(n)
    if m:
        k = int(m.group(1))
        if k <= 0:
            raise ValueError(f"Position k must be greater than 0: {k}")
        return EvaluatorType(f"PRECISION@{k}:{m.group(2)}", m.group(2), k)
    m = _AUC_TAG.fullmatch(n)
    if m:
        return EvaluatorType(f"AUC:{m.group(1)}", m.group(1))
    up = n.upper()
    if up in SIMPLE_TYPES:
        return EvaluatorType(up)
    raise ValueError(f"Unsupported evaluator type: {name}")


def build_evaluator(etype, labels, offsets=None, weights=None, id_tags: Optional[dict] = None, device=None):
    """EvaluatorFactory.buildEvaluator."""
    if isinstance(etype, str):
        etype = parse_evaluator_type(etype)
    simple = {"AUC": AUCEvaluator, "RMSE": RMSEEvaluator, "LOGISTIC_LOSS": LogisticLossEvaluator,
              "POISSON_LOSS": PoissonLossEvaluator, "SMOOTHED_HINGE_LOSS": SmoothedHingeLossEvaluator,
              "SQUARED_LOSS": SquaredLossEvaluator}
    if not etype.is_multi:
        return simple[etype.name](labels, offsets, weights, device)
    if id_tags is None or etype.id_tag not in id_tags:
        raise ValueError(f"id tag {etype.id_tag} required by evaluator {etype.name} not present in the data")
    ids = id_tags[etype.id_tag]
    if etype.k is not None:
        return PrecisionAtKMultiEvaluator(etype.k, etype.id_tag, ids, labels, offsets, weights, device)
    return AUCMultiEvaluator(etype.id_tag, ids, labels, offsets, weights, device)


def default_validation_evaluator(task) -> str:
    """GameEstimator.scala:519-540: AUC for logistic/SVM, RMSE for linear, Poisson loss for Poisson."""
    task = TaskType.parse(task)
    return {TaskType.LOGISTIC_REGRESSION: "AUC", TaskType.SMOOTHED_HINGE_LOSS_LINEAR_SVM: "AUC",
            TaskType.LINEAR_REGRESSION: "RMSE", TaskType.POISSON_REGRESSION: "POISSON_LOSS"}[task]


def training_loss_evaluator_type(task) -> str:
    """GameEstimator.scala:437-459."""
    task = TaskType.parse(task)
    return {TaskType.LOGISTIC_REGRESSION: "LOGISTIC_LOSS", TaskType.LINEAR_REGRESSION: "SQUARED_LOSS",
            TaskType.POISSON_REGRESSION: "POISSON_LOSS",
            TaskType.SMOOTHED_HINGE_LOSS_LINEAR_SVM: "SMOOTHED_HINGE_LOSS"}[task]
