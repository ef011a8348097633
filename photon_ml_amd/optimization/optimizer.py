"""Optimizer base class: Photon's outer convergence state machine, box constraints and state tracking.

Reference: ``photon-lib/.../optimization/Optimizer.scala:37-245`` (tolerances from the state at ZERO
coefficients, ``getConvergenceReason`` 136-150, ``optimize`` 172-196), ``OptimizerState.scala``,
``OptimizationStatesTracker.scala:31-102``, ``OptimizationUtils.scala:34-70`` (box projection) and
``util/ConvergenceReason.scala``.

All vectors are fp64 torch tensors that live on the same device as the data shard (HBM on the GPU path): the
optimizer never moves coefficients between host and device (SURVEY C5 "coefficient broadcast" disappears).
"""
from __future__ import annotations

import enum
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch

from ..normalization.context import NormalizationContext, no_normalization
from . import vector_space

# the zero point's gradient norm (tolerance scale) as a cheap upper bound until needed: GLMObjective.zero_state_bound
LAZY_ZERO_GRADIENT = __import__("os").environ.get("PML_LAZY_ZERO_GRADIENT", "1") != "0"


class ConvergenceReason(str, enum.Enum):
    MAX_ITERATIONS = "max iterations reached"
    FUNCTION_VALUES_CONVERGED = "function values converged"
    GRADIENT_CONVERGED = "gradient converged"
    OBJECTIVE_NOT_IMPROVING = "objective is not improving"


@dataclass
class OptimizerState:
    coefficients: torch.Tensor
    loss: float
    gradient: torch.Tensor
    iter: int

    def grad_norm(self) -> float:
        gn = getattr(self, "_grad_norm", None)        # set by an optimizer that already reduced ||g||^2
        return vector_space.vnorm(self.gradient) if gn is None else gn


class OptimizationStatesTracker:
    """Keeps up to ``max_states`` states plus wall-clock times; pretty-prints the Iter/Time/Value/|g| table."""

    def __init__(self, max_states: int = 100):
        self.max_states = max_states
        self._start = time.time()
        self.times: deque = deque()
        self.states: deque = deque()
        self.convergence_reason: Optional[ConvergenceReason] = None

    @property
    def converged(self) -> bool:
        return self.convergence_reason in (
            ConvergenceReason.FUNCTION_VALUES_CONVERGED,
            ConvergenceReason.GRADIENT_CONVERGED,
        )

    def track(self, state: OptimizerState):
        self.times.append(time.time() - self._start)
        # keep a light copy: coefficients stay on device, scalars on host
        self.states.append(OptimizerState(state.coefficients, state.loss, state.gradient, state.iter))
        if len(self.states) >= self.max_states:
            self.times.popleft()
            self.states.popleft()

    def iterations(self) -> int:
        return self.states[-1].iter if self.states else 0

    def __str__(self):
        reason = self.convergence_reason.value if self.convergence_reason else (
            "Optimizer is not converged properly, please check the log for more information")
        lines = [f"Convergence reason: {reason}", f"{'Iter':>10}{'Time(s)':>10}{'Value':>25}{'|Gradient|':>15}"]
        for st, t in zip(self.states, self.times):
            lines.append(f"{st.iter:10d}{t:10.3f}{st.loss:25.8f}{st.grad_norm():15.2e}")
        return "\n".join(lines) + "\n"

    def to_dict(self) -> dict:
        return {
            "convergence_reason": self.convergence_reason.name if self.convergence_reason else None,
            "iterations": [
                {"iter": s.iter, "time_s": t, "value": s.loss, "grad_norm": s.grad_norm()}
                for s, t in zip(self.states, self.times)
            ],
        }


def project_box(w: torch.Tensor, constraints: Optional[Dict[int, Tuple[float, float]]]) -> torch.Tensor:
    """Clamp coefficients to [lower, upper] per index (OptimizationUtils.projectCoefficientsToSubspace)."""
    if not constraints:
        return w
    idx = torch.tensor(list(constraints.keys()), dtype=torch.long, device=w.device)
    lo = torch.tensor([c[0] for c in constraints.values()], dtype=w.dtype, device=w.device)
    hi = torch.tensor([c[1] for c in constraints.values()], dtype=w.dtype, device=w.device)
    out = w.clone()
    out[idx] = torch.minimum(torch.maximum(w[idx], lo), hi)
    return out


class Optimizer:
    """Abstract optimizer. Subclasses implement ``_init`` and ``_run_one_iteration``."""

    needs_hessian = False

    def __init__(
        self,
        tolerance: float,
        max_iterations: int,
        normalization: Optional[NormalizationContext] = None,
        constraints: Optional[Dict[int, Tuple[float, float]]] = None,
        track_state: bool = True,
    ):
        self.tolerance = float(tolerance)
        self.max_iterations = int(max_iterations)
        self.normalization = normalization or no_normalization()
        self.constraints = constraints
        self.track_state = track_state
        self.loss_abs_tol = 0.0
        self.grad_abs_tol = 0.0
        self._gtol_lazy = None     # (upper bound of grad_abs_tol, thunk of the exact ||g(0)||): see start()
        self.current: Optional[OptimizerState] = None
        self.previous: Optional[OptimizerState] = None
        self.tracker: Optional[OptimizationStatesTracker] = None

    # ----------------------------------------------------------------
    def _calculate_state(self, objective, data, w: torch.Tensor, it: int = 0) -> OptimizerState:
        f, g = objective.calculate(data, w)
        return OptimizerState(w, f, g, it)

    def _set_abs_tolerances(self, state: OptimizerState):
        self.loss_abs_tol = state.loss * self.tolerance
        self.grad_abs_tol = state.grad_norm() * self.tolerance

    def _update_current(self, state: OptimizerState):
        if self.tracker is not None and (self.current is None or state is not self.current):
            self.tracker.track(state)
        self.previous = self.current
        self.current = state

    def convergence_reason(self) -> Optional[ConvergenceReason]:
        cur, prev = self.current, self.previous
        if cur is None:
            return None
        if cur.iter >= self.max_iterations:
            return ConvergenceReason.MAX_ITERATIONS
        if prev is not None and cur.iter == prev.iter:
            return ConvergenceReason.OBJECTIVE_NOT_IMPROVING
        if prev is not None and abs(cur.loss - prev.loss) <= self.loss_abs_tol:
            return ConvergenceReason.FUNCTION_VALUES_CONVERGED
        if self._gtol_lazy is not None:
            if cur.grad_norm() > self._gtol_lazy[0]:
                return None                    # above even the bound: the exact tolerance cannot be met
            self._resolve_grad_tol()
        if cur.grad_norm() <= self.grad_abs_tol:
            return ConvergenceReason.GRADIENT_CONVERGED
        return None

    def _resolve_grad_tol(self):
        """The exact ||g(0)|| tolerance (one transpose pass at the zero point), computed the first time a
        gradient norm falls below the bound."""
        if self._gtol_lazy is not None:
            self.grad_abs_tol = self._gtol_lazy[1]() * self.tolerance
            self._gtol_lazy = None

    def is_done(self) -> bool:
        return self.convergence_reason() is not None

    def clear_inner_state(self):
        self.current = None
        self.previous = None
        self.tracker = OptimizationStatesTracker() if self.track_state else None

    # ----------------------------------------------------------------
    def start(self, objective, data, initial: torch.Tensor, skip_zero_tolerance_pass: bool = False):
        """Set tolerances and the initial state (first half of ``Optimizer.optimize``)."""
        w0 = self.normalization.model_to_transformed_space(initial.to(torch.float64))
        self.clear_inner_state()
        zero_state = None
        self._gtol_lazy = None
        lazy = None
        if not (skip_zero_tolerance_pass and vector_space.current().all_zero(w0)):
            # the zero point first, so the data's margin cache ends at w0 (the first line search then needs no
            # extra forward pass); tagged so a data backend can evaluate it without a pass over the non-zeros
            z = torch.zeros_like(w0)
            z._pml_zero = True
            bound = getattr(objective, "zero_state_bound", None) if LAZY_ZERO_GRADIENT else None
            lazy = bound(data, z) if bound is not None else None
            if lazy is None:
                zero_state = self._calculate_state(objective, data, z)
        init_state = self._calculate_state(objective, data, w0)
        if lazy is not None:
            # f(0) exactly (elementwise pass); ||g(0)|| only as an upper bound until a gradient norm comes close
            # (the transpose pass at the zero point is then paid once, if ever): identical convergence decisions
            f0, gbound, exact = lazy
            self.loss_abs_tol = f0 * self.tolerance
            self.grad_abs_tol = 0.0
            self._gtol_lazy = (gbound * self.tolerance, exact)
        else:
            self._set_abs_tolerances(init_state if zero_state is None else zero_state)
        self._init(objective, data, init_state)
        self._update_current(init_state)
        return init_state

    def step(self, objective, data) -> OptimizerState:
        """Run one optimizer iteration from the current state."""
        from ..utils.timing import trace_range
        with trace_range(f"{type(self).__name__} iteration {self.current.iter + 1}"):
            self._update_current(self._run_one_iteration(objective, data, self.current))
        return self.current

    def optimize(self, objective, data, initial: torch.Tensor, skip_zero_tolerance_pass: bool = False):
        """Minimise ``objective`` over ``data`` from ``initial`` (ORIGINAL space).

        Returns ``(coefficients_in_transformed_space, final_value)`` like ``Optimizer.optimize``.
        ``skip_zero_tolerance_pass`` reuses the initial state for the tolerances when ``initial`` is zero (the
        reference evaluates the same zero point twice on cold start, Appendix C.7); the results are identical.
        """
        self.start(objective, data, initial, skip_zero_tolerance_pass)
        while True:
            self.step(objective, data)
            if self.is_done():
                break
        if self.tracker is not None:
            self.tracker.convergence_reason = self.convergence_reason()
        return self.current.coefficients, self.current.loss

    # checkpoint / resume ---------------------------------------------
    def state_dict(self) -> dict:
        """Everything needed to continue the run bitwise-identically (SURVEY §5 checkpoint: coefficients,
        L-BFGS history, TRON trust radius, tolerances). Tensors stay on their device; ``utils.checkpoint``
        serialises with safetensors."""
        def st(s: Optional[OptimizerState]):
            return None if s is None else {"coefficients": s.coefficients, "loss": s.loss, "gradient": s.gradient,
                                           "iter": s.iter}
        self._resolve_grad_tol()
        return {"kind": type(self).__name__, "loss_abs_tol": self.loss_abs_tol, "grad_abs_tol": self.grad_abs_tol,
                "current": st(self.current), "previous": st(self.previous), "inner": self._inner_state()}

    def load_state_dict(self, sd: dict):
        if sd["kind"] != type(self).__name__:
            raise ValueError(f"checkpoint of a {sd['kind']} cannot resume a {type(self).__name__}")
        self.clear_inner_state()
        self._gtol_lazy = None
        self.loss_abs_tol, self.grad_abs_tol = sd["loss_abs_tol"], sd["grad_abs_tol"]
        mk = lambda d: None if d is None else OptimizerState(d["coefficients"], d["loss"], d["gradient"], d["iter"])
        self.previous, self.current = mk(sd["previous"]), mk(sd["current"])
        self._load_inner_state(sd["inner"])

    def _inner_state(self) -> dict:
        return {}

    def _load_inner_state(self, d: dict):
        pass

    # hooks -----------------------------------------------------------
    def _init(self, objective, data, state: OptimizerState):
        raise NotImplementedError

    def _run_one_iteration(self, objective, data, state: OptimizerState) -> OptimizerState:
        raise NotImplementedError
