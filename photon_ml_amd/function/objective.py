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

    def zero_state_bound(self, data, z: torch.Tensor):
        """(f(0), an upper bound of ||g(0)||, thunk of the exact ||g(0)||) from one elementwise pass, or None when
        the backend cannot bound it (``zero_point_sums``). The optimizer scales its tolerances by f(0) and ||g(0)||
        (Optimizer.scala, Appendix C.7); ||g(0)|| needs a transpose pass, but it is only compared with later
        gradient norms, so a bound decides every iteration whose gradient is above it. g(0) = a (X^T c - s S)
        with c = w l'(offsets), so ||g(0)|| <= max|a| (||X||_F ||c|| + ||s|| |S|)."""
        fn = getattr(data, "zero_point_sums", None)
        if fn is None:
            return None
        norm = self.normalization
        _, shift = norm.effective(z)
        try:
            F, S, csq, xsq = fn(self.loss, shift)
        except AttributeError:              # a wrapper whose local backend cannot bound it
            return None
        b = (xsq * csq) ** 0.5
        if norm.shifts is not None:
            b += float(torch.linalg.vector_norm(norm.shifts.to(torch.float64))) * abs(S)
        if norm.factors is not None:
            b *= float(norm.factors.to(torch.float64).abs().max())
        b = b * (1.0 + 1e-6) + 1e-300             # rounding of the sums: stay an upper bound
        self.n_value_grad += 1

        def exact():
            return float(torch.linalg.vector_norm(self.calculate(data, z)[1].to(torch.float64)))
        return F, b, exact

    def margin_line_search(self, data, x0: torch.Tensor, d: torch.Tensor, t0: float = 1.0,
                           dots=None, ls_opts: Optional[dict] = None) -> Optional["MarginLineSearch"]:
        """Line search along x0 + t d in MARGIN space (GLM margins are affine in t), or None when the data
        backend cannot cache margins. ``dots``: (x0.x0, x0.d, d.d) when the caller already has them.
        ``ls_opts``: extra keywords of the backend's ``ls_begin`` (a speculative pass, see
        ``DeviceGLMData.ls_begin``). See :class:`MarginLineSearch`."""
        if not hasattr(data, "ls_begin"):
            return None
        norm = self.normalization
        w0_eff, shift0 = norm.effective(x0)
        d_eff = d * norm.factors.to(d) if norm.factors is not None else d
        d_shift = -float(torch.dot(d_eff, norm.shifts.to(d_eff))) if norm.shifts is not None else 0.0
        if not data.ls_begin(w0_eff, shift0, d_eff, d_shift, t0, self.loss, **(ls_opts or {})):
            return None
        return MarginLineSearch(self, data, x0, d, dots)

    # ---- TRON trial point from margins (see DeviceGLMData.step_begin) ----------------------------------------
    def step_begin(self, data, w: torch.Tensor) -> bool:
        """Start tracking the margins of a step from ``w``; False when the backend cannot."""
        if not hasattr(data, "step_begin"):
            return False
        w_eff, shift = self.normalization.effective(w)
        return bool(data.step_begin(w_eff, shift))

    def step_add(self, data, alpha: float):
        """The step grew by ``alpha`` times the direction of the last :meth:`hessian_vector` call."""
        data.step_add(alpha)

    def calculate_step(self, data, w_new: torch.Tensor) -> Tuple[float, torch.Tensor]:
        """:meth:`calculate` at ``w_new`` = w + (tracked step), from margins: no forward pass."""
        self.n_value_grad += 1
        norm = self.normalization
        w_eff, shift = norm.effective(w_new)
        f, s, g = data.ls_finish_sums(self.loss, 1.0, w_eff, shift, norm.shifts is not None)
        grad = norm.finalize_vector(g, s)
        if self.l2_weight > 0:
            f += self.l2_value(w_new)
            grad = grad + self.l2_weight * w_new
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


DEFERRED_DOTS = object()   # ``dots`` sentinel: the caller assigns (a, b, c) itself before the first eval
# trial steps evaluated together once a line search needs a second trial (1: one pass per trial). Off by default:
# measured on game5pl (profiles/lbfgs_plans_r6.md) the 6-step pass costs 0.97 ms -- the fp64 logistic loss at six
# margins per row is compute-bound -- and L-BFGS's first search then still needed three zoom trials.
LS_LADDER = int(__import__("os").environ.get("PML_LS_LADDER", "1"))


class MarginLineSearch:
    """phi(t) = F(x0 + t d) for a GLM objective, evaluated from cached margins.

    z(t) = z0 + t zd with z0 the margins at x0 (kept by the last full evaluation) and zd = X d_eff + d_shift (one
    forward pass), so each trial costs one elementwise pass over the rows (``ls_eval_kernel``) instead of a
    forward + transpose pass over every non-zero; phi'(t) = sum w l'(z(t)) zd + l2 x(t).d (the normalization
    shift terms cancel: d_eff . G - S d_eff . s = sum w l' (zd - d_shift) + S d_shift). Only the ACCEPTED step
    pays the transpose pass for the full gradient. The reference evaluates the full objective (broadcast +
    treeAggregate) at every trial point (Breeze StrongWolfeLineSearch through ``DiffFunction.calculate``).
    """

    def __init__(self, obj: GLMObjective, data, x0: torch.Tensor, d: torch.Tensor, dots=None):
        from ..optimization.vector_space import vdots
        self.obj, self.data, self.x0, self.d = obj, data, x0, d
        l2 = obj.l2_weight
        self.l2 = l2
        self._trials = {}
        self._n_eval = 0
        if l2 > 0 and dots is not DEFERRED_DOTS:
            self.a, self.b, self.c = dots if dots is not None else vdots([(x0, x0), (x0, d), (d, d)])

    def eval(self, t: float):
        """phi(t), phi'(t). From the second trial on, a backend with ``ls_eval_many`` evaluates the strong Wolfe
        search's whole extrapolation ladder t, 1.5 t, 2.25 t, ... (LS_LADDER steps) in one pass and one readback:
        a first step that is too short (L-BFGS's first iteration, t0 = 1 / ||d||) then costs one pass, not one
        pass and one host round trip per trial. Same values as trial-by-trial evaluation (bitwise)."""
        self._n_eval += 1
        t = float(t)
        got = self._trials.get(t)
        if got is None:
            many = getattr(self.data, "ls_eval_many", None)
            if many is not None and LS_LADDER > 1 and self._n_eval > 1:
                from ..optimization.line_search import EXTRAPOLATION
                ts = [t]
                for _ in range(LS_LADDER - 1):
                    ts.append(ts[-1] * EXTRAPOLATION)
                for tk, v in zip(ts, many(self.obj.loss, ts)):
                    self._trials[tk] = v
                got = self._trials[t]
            else:
                got = self.data.ls_eval(self.obj.loss, t)
        f, dd = got
        return self.adjust(f, dd, t)

    def adjust(self, f: float, dd: float, t: float):
        """phi(t) and phi'(t) from the data terms (F, D) at t: the L2 terms from the cached inner products."""
        if self.l2 > 0:
            f += 0.5 * self.l2 * (self.a + 2.0 * t * self.b + t * t * self.c)
            dd += self.l2 * (self.b + t * self.c)
        return f, dd

    def finish(self, t: float):
        """(x(t), f(x(t)), gradient at x(t)) — one transpose pass. With a backend that keeps the sums on the
        device (``ls_finish_device``) f is a 0-d device tensor: the caller reads it together with its next
        synchronisation (L-BFGS: the history pair's scalars), not right after the transpose pass."""
        norm = self.obj.normalization
        fused = getattr(self.data, "ls_finish_fused", None)
        if (fused is not None and norm.factors is None and norm.shifts is None and self.x0.is_cuda
                and self.x0.dtype == self.d.dtype == torch.float64 and self.x0.is_contiguous()
                and self.d.is_contiguous()):
            # the step, the transpose pass and the gradient epilogue (g + l2 x) with one launch after the pass
            x, f, grad = fused(self.obj.loss, t, self.x0, self.d, self.obj.l2_weight)
            self.obj.n_value_grad += 1
            if self.obj.l2_weight > 0:
                f = f + 0.5 * self.l2 * (self.a + 2.0 * t * self.b + t * t * self.c)
            return x, f, grad
        x = self.x0 + t * self.d
        w_eff, shift = norm.effective(x)
        fin = getattr(self.data, "ls_finish_device", None)
        if fin is not None:
            f, s, g = fin(self.obj.loss, t, w_eff, shift, norm.shifts is not None)
        else:
            f, s, g = self.data.ls_finish_sums(self.obj.loss, t, w_eff, shift, norm.shifts is not None)
        self.obj.n_value_grad += 1
        grad = norm.finalize_vector(g, s)
        if self.obj.l2_weight > 0:
            # ||x0 + t d||^2 from the cached inner products (no host synchronisation)
            f += 0.5 * self.l2 * (self.a + 2.0 * t * self.b + t * t * self.c)
            grad = grad + self.obj.l2_weight * x
        return x, f, grad

