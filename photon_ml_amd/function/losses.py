"""Pointwise GLM loss functions l(z, y), dl/dz and d2l/dz2 on torch tensors.

Every loss is elementwise and vectorised; the same code runs on CPU (fp64 reference path) and on the GPU
(torch fallbacks for small problems). The HIP kernels in ``photon_ml_amd/ops/csrc`` implement the same
formulas in their fused epilogues (loss ids below must match ``LossId`` in ``glm_kernels.hip``).

Reference formulas:
  * logistic  ``photon-api/.../function/glm/LogisticLossFunction.scala:45-90``
  * poisson   ``photon-api/.../function/glm/PoissonLossFunction.scala:31-53``
  * squared   ``photon-api/.../function/glm/SquaredLossFunction.scala:32-55``
  * smoothed hinge ``photon-api/.../function/svm/SmoothedHingeLossFunction.scala:30-85``
  * log1pExp  ``photon-lib/.../util/MathUtils.scala:22-49``
"""
from __future__ import annotations

import math

import torch

from ..constants import POSITIVE_RESPONSE_THRESHOLD, TaskType


def log1p_exp(x: torch.Tensor) -> torch.Tensor:
    """Numerically stable log(1 + exp(x)) (== softplus)."""
    return torch.where(x > 0, x + torch.log1p(torch.exp(-x.abs())), torch.log1p(torch.exp(-x.abs())))


def log1p_exp_scalar(x: float) -> float:
    return x + math.log1p(math.exp(-x)) if x > 0 else math.log1p(math.exp(x))


class PointwiseLoss:
    """Base class. ``loss_id`` is shared with the HIP kernels."""

    name = "base"
    loss_id = -1
    twice_differentiable = True

    def loss_and_dz(self, z: torch.Tensor, y: torch.Tensor):  # pragma: no cover - abstract
        raise NotImplementedError

    def dzz(self, z: torch.Tensor, y: torch.Tensor) -> torch.Tensor:  # pragma: no cover - abstract
        raise NotImplementedError

    def __repr__(self):
        return f"{type(self).__name__}()"


class LogisticLoss(PointwiseLoss):
    name = "logistic"
    loss_id = 0

    def loss_and_dz(self, z, y):
        pos = y > POSITIVE_RESPONSE_THRESHOLD
        loss = torch.where(pos, log1p_exp(-z), log1p_exp(z))
        sig = torch.sigmoid(z)
        # -sigmoid(-z) = sigmoid(z) - 1
        dz = torch.where(pos, sig - 1.0, sig)
        return loss, dz

    def dzz(self, z, y):
        s = torch.sigmoid(z)
        return s * (1.0 - s)


class PoissonLoss(PointwiseLoss):
    name = "poisson"
    loss_id = 1

    def loss_and_dz(self, z, y):
        e = torch.exp(z)
        return e - y * z, e - y

    def dzz(self, z, y):
        return torch.exp(z)


class SquaredLoss(PointwiseLoss):
    name = "squared"
    loss_id = 2

    def loss_and_dz(self, z, y):
        d = z - y
        return 0.5 * d * d, d

    def dzz(self, z, y):
        return torch.ones_like(z)


class SmoothedHingeLoss(PointwiseLoss):
    """Rennie & Srebro smoothed hinge. Differentiable once; no Hessian (TRON unsupported)."""

    name = "smoothed_hinge"
    loss_id = 3
    twice_differentiable = False

    def loss_and_dz(self, z, y):
        yy = torch.where(y < POSITIVE_RESPONSE_THRESHOLD, -1.0, 1.0).to(z.dtype)
        t = yy * z
        loss = torch.where(t <= 0, 0.5 - t, torch.where(t < 1, 0.5 * (1 - t) * (1 - t), torch.zeros_like(t)))
        d = torch.where(t < 0, -torch.ones_like(t), torch.where(t < 1, t - 1.0, torch.zeros_like(t)))
        return loss, d * yy

    def dzz(self, z, y):
        raise NotImplementedError("smoothed hinge loss is not twice differentiable")


LOGISTIC = LogisticLoss()
POISSON = PoissonLoss()
SQUARED = SquaredLoss()
SMOOTHED_HINGE = SmoothedHingeLoss()

_BY_TASK = {
    TaskType.LOGISTIC_REGRESSION: LOGISTIC,
    TaskType.POISSON_REGRESSION: POISSON,
    TaskType.LINEAR_REGRESSION: SQUARED,
    TaskType.SMOOTHED_HINGE_LOSS_LINEAR_SVM: SMOOTHED_HINGE,
}


def loss_for_task(task) -> PointwiseLoss:
    task = TaskType.parse(task)
    if task not in _BY_TASK:
        raise ValueError(f"no loss for task {task}")
    return _BY_TASK[task]
