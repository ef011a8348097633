"""TRON: trust-region Newton with truncated conjugate gradient (LIBLINEAR-style).

Reference: ``photon-lib/.../optimization/TRON.scala:80-340`` — constants eta=(1e-4, .25, .75),
sigma=(.25, .5, 4); delta0 = ||g0||, first-iteration ``delta = min(delta, ||step||)``; CG at most 20 iterations
with tolerance ``0.1 ||g||`` and trust-region boundary handling; accept if actual > eta0 * predicted; at most 5
consecutive improvement failures; defaults tol 1e-5, maxIter 15.

MI355X-native difference: every Hessian-vector product in one outer iteration is taken at the SAME point w, so
the data backend caches ``wt_i l''(z_i)`` once per outer iteration (K2 in SURVEY §2.8) instead of re-computing
margins in each CG step as the reference does (``HessianVectorAggregator.scala:111``).
"""
from __future__ import annotations

import logging
import math
import os

import torch

from .optimizer import Optimizer, OptimizerState, project_box
from .vector_space import vdot as _dot, vnorm as _norm

DEFAULT_MAX_NUM_FAILURE = 5
DEFAULT_TOLERANCE = 1.0e-5
DEFAULT_MAX_ITER = 15
MAX_CG_ITERATIONS = 20
# Evaluate each trial point w + s from margins accumulated during CG (GLMObjective.step_begin) instead of a full
# forward pass; the data backend must support it (device / torch reference backends), otherwise ignored.
MARGIN_TRIAL = os.environ.get("PML_TRON_MARGIN_TRIAL", "1") != "0"

log = logging.getLogger(__name__)


class TRON(Optimizer):
    needs_hessian = True
    eta0, eta1, eta2 = 1e-4, 0.25, 0.75
    sigma1, sigma2, sigma3 = 0.25, 0.5, 4.0

    def __init__(self, normalization=None, max_num_failures: int = DEFAULT_MAX_NUM_FAILURE,
                 tolerance: float = DEFAULT_TOLERANCE, max_iterations: int = DEFAULT_MAX_ITER,
                 constraints=None, track_state: bool = True):
        super().__init__(tolerance, max_iterations, normalization, constraints, track_state)
        self.max_num_failures = max_num_failures
        self.margin_trial = MARGIN_TRIAL
        self.delta = float("inf")
        self.total_cg_iterations = 0

    def clear_inner_state(self):
        super().clear_inner_state()
        self.delta = float("inf")
        self.total_cg_iterations = 0

    def _init(self, objective, data, state):
        self.delta = state.grad_norm()

    def _inner_state(self) -> dict:
        return {"delta": self.delta, "total_cg_iterations": self.total_cg_iterations}

    def _load_inner_state(self, d: dict):
        self.delta, self.total_cg_iterations = d["delta"], d["total_cg_iterations"]

    @staticmethod
    def truncated_cg(objective, data, w, gradient, delta, track=None):
        """``track(alpha)``: called after each step update ``step += alpha * direction`` (net alpha on the trust
        region boundary) right after the Hessian-vector product of that direction (margin-space trial)."""
        step = torch.zeros_like(gradient)
        residual = -gradient
        direction = residual.clone()
        cg_tol = 0.1 * _norm(gradient)
        it = 0
        rtr = _dot(residual, residual)
        while it < MAX_CG_ITERATIONS:
            if math.sqrt(max(rtr, 0.0)) <= cg_tol:
                break
            it += 1
            hd = objective.hessian_vector(data, w, direction)
            alpha = rtr / _dot(direction, hd)
            step = step + alpha * direction
            if _norm(step) > delta:
                step = step - alpha * direction
                std = _dot(step, direction)
                sts = _dot(step, step)
                dtd = _dot(direction, direction)
                dsq = delta * delta
                rad = math.sqrt(max(std * std + dtd * (dsq - sts), 0.0))
                if std >= 0:
                    alpha = (dsq - sts) / (std + rad)
                else:
                    alpha = (rad - std) / dtd
                step = step + alpha * direction
                if track is not None:
                    track(alpha)          # step = previous step + alpha * direction
                residual = residual - alpha * hd
                break
            if track is not None:
                track(alpha)
            residual = residual - alpha * hd
            rnew = _dot(residual, residual)
            beta = rnew / rtr
            direction = residual + beta * direction
            rtr = rnew
        return it, step, residual

    def _run_one_iteration(self, objective, data, state: OptimizerState) -> OptimizerState:
        w = state.coefficients
        f_prev, g_prev = state.loss, state.gradient
        first = state.iter == 0
        failures = 0
        while failures < self.max_num_failures:
            margins = self.margin_trial and hasattr(objective, "step_begin") and objective.step_begin(data, w)
            track = (lambda a: objective.step_add(data, a)) if margins else None
            cg_iter, step, residual = self.truncated_cg(objective, data, w, g_prev, self.delta, track)
            self.total_cg_iterations += cg_iter
            w_new = w + step
            gs = _dot(g_prev, step)
            predicted = -0.5 * (gs - _dot(step, residual))
            if margins:   # margins(w + step) = z(w) + sum alpha_i X d_i: elementwise loss + transpose pass only
                f_new, g_new = objective.calculate_step(data, w_new)
            else:
                f_new, g_new = objective.calculate(data, w_new)
            actual = f_prev - f_new
            step_norm = _norm(step)
            if first:
                self.delta = min(self.delta, step_norm)
            denom = f_new - f_prev - gs
            alpha = self.sigma3 if denom <= 0 else max(self.sigma1, -0.5 * (gs / denom))
            if actual < self.eta0 * predicted:
                self.delta = min(max(alpha, self.sigma1) * step_norm, self.sigma2 * self.delta)
            elif actual < self.eta1 * predicted:
                self.delta = max(self.sigma1 * self.delta, min(alpha * step_norm, self.sigma2 * self.delta))
            elif actual < self.eta2 * predicted:
                self.delta = max(self.sigma1 * self.delta, min(alpha * step_norm, self.sigma3 * self.delta))
            else:
                self.delta = max(self.delta, min(alpha * step_norm, self.sigma3 * self.delta))
            log.debug("iter %d act %.3e pre %.3e delta %.3e f %.3e |g| %.3e CG %d",
                      state.iter, actual, predicted, self.delta, f_new, _norm(g_new), cg_iter)
            if actual > self.eta0 * predicted:
                return OptimizerState(project_box(w_new, self.constraints), f_new, g_new, state.iter + 1)
            failures += 1
        return state
