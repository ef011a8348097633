"""GLM objective functions: loss aggregate + normalisation folding + L2 regularisation.

Reference:
  * ``ObjectiveFunction`` / ``DiffFunction`` / ``TwiceDiffFunction`` traits:
    ``photon-lib/.../function/{ObjectiveFunction,DiffFunction,TwiceDiffFunction}.scala``.
  * L2 mix-ins (value ``+ l2/2 ||w||^2``, gradient ``+ l2 w``, Hv ``+ l2 v``, Hdiag ``+ l2``; the intercept is
    regularised too): ``photon-lib/.../function/L2Regularization.scala:25-184``.
  * Distributed/single-node GLM loss: ``photon-api/.../function/glm/{Distributed,SingleNode}GLMLossFunction.scala``.
    Here one class serves both: the ``data`` argument is any :class:`GLMComputable` (local shard, device shard,
    or a distributed wrapper that all-reduces over RCCL), so the "distributed vs single node" split of the
    reference collapses into the data backend.
  * Smoothed hinge: the reference ignores normalisation for this loss
    (``SmoothedHingeLossFunction.scala:73-84``). We deliberately FIX that quirk: the same
    effective-coefficient folding is applied for every loss, so models trained with normalisation are correct in
    the original space.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from ..normalization.context import NormalizationContext, no_normalization
from .losses import PointwiseLoss


class GLMObjective:
    """Objective F(w) = sum_i wt_i l(z_i, y_i) + l2/2 ||w||^2 in the (normalised) transformed space."""

    def __init__(
        self,
        loss: PointwiseLoss,
        l2_weight: float = 0.0,
        normalization: Optional[NormalizationContext] = None,
    ):
        self.loss = loss
        self.l2_weight = float(l2_weight)
        self.normalization = normalization or no_normalization()
        # evaluation counters (observability; the reference logs these through Timed blocks)
        self.n_value_grad = 0
        self.n_hv = 0

    @property
    def twice_differentiable(self) -> bool:
        return self.loss.twice_differentiable

    def with_l2(self, l2_weight: float) -> "GLMObjective":
        return GLMObjective(self.loss, l2_weight, self.normalization)

    # ------------------------------------------------------------------
    def l2_value(self, w: torch.Tensor) -> float:
        return 0.5 * self.l2_weight * float(torch.dot(w, w)) if self.l2_weight > 0 else 0.0

    def calculate(self, data, w: torch.Tensor) -> Tuple[float, torch.Tensor]:
        """Value and gradient at ``w`` (transformed space)."""
        self.n_value_grad += 1
        norm = self.normalization
        w_eff, shift = norm.effective(w)
        f, s, g = data.value_grad_sums(self.loss, w_eff, shift)
        grad = norm.finalize_vector(g, s)
        if self.l2_weight > 0:
            f += self.l2_value(w)
            grad = grad + self.l2_weight * w
        return f, grad

    def value(self, data, w: torch.Tensor) -> float:
        return self.calculate(data, w)[0]

    def gradient(self, data, w: torch.Tensor) -> torch.Tensor:
        return self.calculate(data, w)[1]

    def hessian_vector(self, data, w: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
        if not self.twice_differentiable:
            raise NotImplementedError(f"{self.loss} has no Hessian")
        self.n_hv += 1
        norm = self.normalization
        w_eff, shift = norm.effective(w)
        v_eff = v * norm.factors.to(v) if norm.factors is not None else v
        v_shift = float(torch.dot(v_eff, norm.shifts.to(v_eff))) if norm.shifts is not None else 0.0
        h, p = data.hv_sums(self.loss, w_eff, shift, v_eff, v_shift)
        hv = norm.finalize_vector(h, p)
        if self.l2_weight > 0:
            hv = hv + self.l2_weight * v
        return hv

    def hessian_diagonal(self, data, w: torch.Tensor) -> torch.Tensor:
        """Raw-coefficient Hessian diagonal (HessianDiagonalAggregator ignores normalisation: Appendix C.3)."""
        if not self.twice_differentiable:
            raise NotImplementedError(f"{self.loss} has no Hessian")
        d = data.hdiag_sums(self.loss, w)
        if self.l2_weight > 0:
            d = d + self.l2_weight
        return d
