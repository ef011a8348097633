"""L-BFGS and OWL-QN on device-resident fp64 vectors.

Reference adapters: ``photon-lib/.../optimization/LBFGS.scala:39-156`` (defaults maxIter 100, m 10, tol 1e-7;
box projection after each step, 70-75) and ``OWLQN.scala:40-86`` (constant per-coordinate L1 weight). The
reference wraps Breeze; here the quasi-Newton engine is native to this framework:

* two-loop recursion (K16 of SURVEY §2.8) over an ``m``-deep history of (s, y) pairs kept as one [2m, D] device
  buffer (one allocation, no per-iteration mallocs), initial scaling ``s.y / y.y`` of the newest pair;
* strong-Wolfe line search, first step ``1/||d||`` then 1 (Breeze's choice);
* OWL-QN (K17): pseudo-gradient, direction sign correction, orthant-projected steps, backtracking line search
  (shrink 0.1 on the first iteration then 0.5), L1 added to the reported value and gradient, exactly as the
  reference reports ``adjustedValue``/``adjustedGradient`` to the outer state machine;
* history reset on a failed line search, give-up (ObjectiveNotImproving) on a second consecutive failure.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from .line_search import LineSearchFailed, backtracking, strong_wolfe
from . import vector_space
from .optimizer import Optimizer, OptimizerState, project_box
from .vector_space import vdot as _dot, vnorm as _norm

DEFAULT_MAX_ITER = 100
# L-BFGS line searches in margin space when the data backend caches margins (GLMObjective.margin_line_search)
MARGIN_LINE_SEARCH = os.environ.get("PML_MARGIN_LINE_SEARCH", "1") != "0"
# Device vectors at least this long use the vector-free two-loop (one Gram kernel + one sync) instead of 4k + 1
# dependent dot products. Measured neutral on one GPU at D = 1M (42.97 vs 43.13 ms/step on the headline bench: the
# dot-product recursion is ~2 % of an iteration), so off by default for replicated vectors; feature-sharded
# vectors always use it (one all-reduce instead of 4k + 1).
GRAM_MIN_DIM = int(os.environ.get("PML_LBFGS_GRAM_MIN_DIM", str(1 << 62)))
# Replicated device vectors run the two-loop with 0-d device scalars (PML_LBFGS_DEVICE_TWO_LOOP=0: host scalars,
# one synchronisation per dot product).
DEVICE_TWO_LOOP = os.environ.get("PML_LBFGS_DEVICE_TWO_LOOP", "1") != "0"
# New history pair (s, y, s.y, y.y, 1/s.y, s.y/y.y, g.g) in one HIP kernel + one synchronisation. (A cooperative
# single-launch two-loop kernel was measured SLOWER than the torch recursion below: 20 grid barriers at ~25 us
# each, 0.61 ms per direction vs ~0.2 ms; profiles/lbfgs_device_two_loop_ab.md.)
NATIVE_PAIR = os.environ.get("PML_LBFGS_NATIVE_PAIR", "1") != "0"
# queue the NEXT iteration's two-loop direction (with the new pair, as if accepted) before the pair's host
# synchronisation: the GPU computes it while the host runs the curvature / convergence bookkeeping
SPECULATE_DIRECTION = os.environ.get("PML_LBFGS_SPECULATE", "1") != "0"
# ... and also queue that direction's margin pass (the margin line search's first trial) before the synchronisation,
# so the GPU never waits for the host between two iterations; skipped when the next iteration cannot run
# (max_iterations), discarded when the pair is rejected or the data ran another pass in between
SPECULATE_MARGINS = os.environ.get("PML_LBFGS_SPECULATE_MARGINS", "1") != "0"
# ... only while the last loss drop exceeds this multiple of the loss tolerance (else the iteration likely stops on
# the tolerance and the queued pass is wasted)
SPECULATE_LOSS_MARGIN = float(os.environ.get("PML_LBFGS_SPECULATE_LOSS_MARGIN", "20"))
# Whole-iteration plans: with the margin line search on a device backend, an iteration's direction, its margin pass,
# the gradient at the first trial step t = 1 and its history pair are queued as one chain, with two readbacks: A
# (the line-search scalars, right after the margin pass) and B (the pair's scalars). The host validates t = 1 on A
# while the GPU already runs the speculative gradient pass, queues the NEXT iteration's chain, and only then waits
# for B: the GPU does not wait for the host between the passes or between iterations. A plan is used only when the
# strong-Wolfe search accepts t = 1 at its first trial and the pair passes the curvature test -- the decisions the
# unplanned iteration takes, on the same values, so the iterates are bitwise those of PML_LBFGS_PLAN=0. Otherwise
# the data backend's margin state is restored (``ls_restore``: a speculative pass writes the other buffer pair) and
# the iteration runs the ordinary search from the plan's direction pass (a rejected t = 1 wastes one gradient pass).
# Off by default: on game5pl the planned fixed-effect update ran 30.5 instead of 31.5 ms inside a profiled window
# (97.8 % busy, idle gaps 1.38 -> 0.65 ms), but end to end it was no faster (FE 32.4 / 33.2 vs 32.1 / 32.2 ms bf16,
# 52.9 vs 52.5 fp64): each rejected t = 1 (6 of 115 plans) wastes a gradient pass (profiles/lbfgs_plans_r6.md).
PLAN = os.environ.get("PML_LBFGS_PLAN", "0") != "0"
PLAN_TEST_REJECT = 0        # tests only: treat every n-th planned step as rejected (exercises the fallback)
# Gated first-trial finish (iterations > 0, margin line search on a device backend): the strong-Wolfe decision on the
# first trial t = 1 is also taken on the device, right after the direction pass, and the gradient pass at that step
# is queued behind it, gated on the decision (its workgroups exit when the step is rejected): the GPU does not wait
# for the host's round trip between the two passes, and a rejection costs no pass. The host reads [pre, F, D, device
# decision] once, decides on the same values itself and uses the gated results only when both accept. Off by default:
# bitwise the host-decided iterates, but end to end no faster on game5pl (FE bf16 32.39 / 31.98 vs 32.27 / 31.93 ms,
# fp64 51.67 vs 52.23; profiles/lbfgs_plans_r6.md).
GATED_FINISH = os.environ.get("PML_LBFGS_GATED", "0") != "0"
GATED_TEST_DISAGREE = False   # tests only: pretend the device rejected every gated step (exercises the restore)
# Two-loop as 2k + 1 fused HIP step kernels launched from C++ (no Python between launches); 0: torch recursion
NATIVE_TWO_LOOP = os.environ.get("PML_LBFGS_NATIVE_TWO_LOOP", "1") != "0"
# Device two-loop method for replicated vectors: "gram" = vector-free recursion on the device (one Gram pass, the
# recursion in one workgroup, one combination pass: 3 launches), "chain" = the 2k + 1 step kernels
TWO_LOOP_METHOD = os.environ.get("PML_LBFGS_TWO_LOOP", "gram")
DEFAULT_NUM_CORRECTIONS = 10
DEFAULT_TOLERANCE = 1.0e-7


def _device_loop(g: torch.Tensor) -> bool:
    """Replicated device vectors: the two-loop keeps its scalars on the device (no host synchronisation)."""
    return g.is_cuda and not vector_space.current().sharded and DEVICE_TWO_LOOP


_PINNED = {}


def _async_host(t: torch.Tensor):
    """Queue a copy of the small device tensor ``t`` into a reused pinned host buffer; returns (buffer, event
    recorded after the copy). The buffer is valid once the event has completed."""
    key = t.device
    buf = _PINNED.get(key)
    if buf is None or buf.numel() < t.numel():
        buf = _PINNED[key] = torch.empty(max(16, t.numel()), dtype=torch.float64, pin_memory=True)
    buf[: t.numel()].copy_(t, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    return buf, ev


_RING = {}


def _pinned_slot(device, n: int = 16) -> torch.Tensor:
    """A pinned host buffer from a small per-device ring (plan readbacks: at most two plans are outstanding)."""
    ring = _RING.get(device)
    if ring is None:
        ring = _RING[device] = [[torch.empty(n, dtype=torch.float64, pin_memory=True) for _ in range(4)], 0]
    bufs, i = ring
    ring[1] = (i + 1) % len(bufs)
    return bufs[i]


class _Plan:
    """Work queued for the iteration that starts at (x, g): direction ``d``, its line-search dots ``pre`` (device
    vector or host list) and ``mls``. A DEEP plan (``deep``) also holds the margin search of ``d`` (``mls``: the
    MarginLineSearch object), the step to t = 1 (``x1``, ``g1``), the history pair (``s``, ``y``, ``out``), the
    readbacks A = [pre (4), (F, D) of the first trial] (``host`` + ``ev_a``) and B = pair scalars (5) (``host[6:]``
    + ``ev``), and the data backend's margin state before the plan (``ck_start``), after its direction pass
    (``ck_fwd``) and after its gradient pass (``ck_fin``). A shallow plan's ``mls`` is (MarginLineSearch, pass
    count) or None, as before."""

    def __init__(self, x, g, d, pre=None, mls=None):
        self.x, self.g, self.d, self.pre, self.mls = x, g, d, pre, mls
        self.deep = False
        self.data = self.passes = self.host = self.ev = self.ev_a = None
        self.x1 = self.g1 = self.s = self.y = self.out = None
        self.ck_start = self.ck_fwd = self.ck_fin = None


class _Unplanned(Exception):
    """The line search wants a trial other than the planned t = 1."""


class _History:
    """Ring buffer of the last m (s, y) pairs plus rho = 1/(s.y) (host floats; for device vectors also 0-d
    device tensors rho_t and the newest pair's scaling s.y / y.y, so the two-loop never synchronises)."""

    def __init__(self, m: int):
        self.m = m
        self.s = []
        self.y = []
        self.rho = []
        self.rho_t = []
        self.gamma_t = None

    def clear(self):
        self.s, self.y, self.rho, self.rho_t, self.gamma_t = [], [], [], [], None

    def push(self, s: torch.Tensor, y: torch.Tensor) -> bool:
        if _device_loop(s):
            # s.y and y.y in ONE host synchronisation (the curvature test is a host decision)
            sy_t, yy_t = torch.dot(s, y), torch.dot(y, y)
            sy, yy = torch.stack([sy_t, yy_t]).tolist()
        else:
            sy_t = yy_t = None
            sy = _dot(s, y)
        if not (sy > 1e-300) or sy != sy:
            return False  # curvature condition violated: skip (Breeze would raise NaNHistory)
        self.s.append(s)
        self.y.append(y)
        self.rho.append(1.0 / sy)
        if sy_t is not None:
            self.rho_t.append(1.0 / sy_t)
            self.gamma_t = sy_t / yy_t
        if len(self.s) > self.m:
            self.s.pop(0)
            self.y.pop(0)
            self.rho.pop(0)
            if self.rho_t:
                self.rho_t.pop(0)
        return True

    def _with_pair(self, s, y, rho_t, gamma_t) -> "_History":
        """A copy of this history with one more (device) pair, for a speculative direction."""
        h = _History(self.m)
        h.s, h.y, h.rho_t = (self.s + [s])[-self.m:], (self.y + [y])[-self.m:], (self.rho_t + [rho_t])[-self.m:]
        h.rho, h.gamma_t = [0.0] * len(h.s), gamma_t
        return h

    def commit(self, s, y, sy: float, rho_t, gamma_t):
        """Append a pair whose scalars are known (host s.y; device 1/s.y and s.y/y.y)."""
        self.s.append(s)
        self.y.append(y)
        self.rho.append(1.0 / sy)
        self.rho_t.append(rho_t)
        self.gamma_t = gamma_t
        if len(self.s) > self.m:
            self.s.pop(0)
            self.y.pop(0)
            self.rho.pop(0)
            self.rho_t.pop(0)

    def push_pair(self, x, x0, g, g0, extra: Optional[torch.Tensor] = None, speculate=None):
        """push(x - x0, g - g0); replicated device vectors: the pair and its scalars in ONE kernel
        (``ops.native.lbfgs_pair``) and one host synchronisation for the curvature test, which also returns
        ||g||^2. ``extra``: a 0-d device scalar read in the same synchronisation (the accepted step's loss, left
        on the device by the margin line search). ``speculate(history_with_pair)``: queued before the
        synchronisation (its result is returned either way: the caller abandons it when the pair is rejected).
        Returns (pushed, ||g||^2 or None, extra as a float or None, speculation or None)."""
        if NATIVE_PAIR and _device_loop(g):
            from ..ops.native import lbfgs_pair
            r = lbfgs_pair(x, x0, g, g0)
            if r is not None:
                s, y, out = r
                src = out if extra is None else torch.cat([out, extra.reshape(1).to(out)])
                # the scalars leave the device BEFORE the speculative work is queued: the host resumes as soon as
                # they are ready and does its bookkeeping while the GPU runs the next direction and margin pass
                host, ev = _async_host(src)
                # the speculative history has device scalars only: it must take the device two-loop
                spec = (speculate(self._with_pair(s, y, out[2], out[3]))
                        if speculate is not None and len(self.rho_t) == len(self.s) else None)
                ev.synchronize()
                vals = host[: src.numel()].tolist()
                sy, yy, _, _, gg = vals[:5]
                ex = vals[5] if extra is not None else None
                if not (sy > 1e-300) or sy != sy:
                    return False, gg, ex, spec
                self.commit(s, y, sy, out[2], out[3])
                return True, gg, ex, spec
        return self.push(x - x0, g - g0), None, (None if extra is None else float(extra)), None

    def _apply_inverse_device(self, g: torch.Tensor, negate: bool = False) -> torch.Tensor:
        """Two-loop with 0-d device scalars, no synchronisation: the fused HIP step-kernel chain
        (``ops.native.two_loop``), else torch dot products + fused scaled adds (same recursion and order)."""
        if NATIVE_TWO_LOOP:
            from ..ops.native import two_loop, two_loop_gram
            q = two_loop_gram(self.s, self.y, g, negate) if TWO_LOOP_METHOD == "gram" else None
            if q is None:
                q = two_loop(self.s, self.y, self.rho_t, self.gamma_t, g, negate)
            if q is not None:
                return q
        return self._apply_inverse_device_torch(g, negate)

    def _apply_inverse_device_torch(self, g: torch.Tensor, negate: bool = False) -> torch.Tensor:
        q = g.clone()
        k = len(self.s)
        alpha = [None] * k
        for i in range(k - 1, -1, -1):
            alpha[i] = self.rho_t[i] * torch.dot(self.s[i], q)
            q.addcmul_(self.y[i], alpha[i], value=-1.0)
        q.mul_(self.gamma_t)
        for i in range(k):
            beta = self.rho_t[i] * torch.dot(self.y[i], q)
            q.addcmul_(self.s[i], alpha[i] - beta)
        return q.neg_() if negate else q

    def apply_inverse(self, g: torch.Tensor, negate: bool = False) -> torch.Tensor:
        """Two-loop recursion: returns H g (-H g with ``negate``)."""
        if self.s and _device_loop(g) and len(self.rho_t) == len(self.s) and g.numel() < GRAM_MIN_DIM:
            return self._apply_inverse_device(g, negate)
        q = self._apply_inverse_host(g)
        return -q if negate else q

    def _apply_inverse_host(self, g: torch.Tensor) -> torch.Tensor:
        if self.s and (vector_space.current().sharded or (g.is_cuda and g.numel() >= GRAM_MIN_DIM)):
            return self._apply_inverse_gram(g)
        q = g.clone()
        k = len(self.s)
        alpha = [0.0] * k
        for i in range(k - 1, -1, -1):
            alpha[i] = self.rho[i] * _dot(self.s[i], q)
            q.add_(self.y[i], alpha=-alpha[i])
        if k > 0:
            yy = _dot(self.y[-1], self.y[-1])
            q.mul_((1.0 / self.rho[-1]) / yy)
        for i in range(k):
            beta = self.rho[i] * _dot(self.y[i], q)
            q.add_(self.s[i], alpha=alpha[i] - beta)
        return q

    def _apply_inverse_gram(self, g: torch.Tensor) -> torch.Tensor:
        """Vector-free two-loop (Chen, Wang & Zhou 2014, "Large-scale L-BFGS using MapReduce"): H g is a linear
        combination of the basis b = [s_0..s_{k-1}, y_0..y_{k-1}, g]; the recursion runs on the (2k+1) coefficient
        vector delta using the Gram matrix B = b b^T, which costs ONE batched all-reduce of (2k+1)^2 scalars per
        iteration over feature shards instead of 4k+1 sequential scalar all-reduces. Exact in exact arithmetic."""
        k = len(self.s)
        basis = self.s + self.y + [g]
        B = vector_space.current().gram(basis)
        delta = torch.zeros(2 * k + 1, dtype=torch.float64)
        delta[2 * k] = 1.0
        alpha = [0.0] * k
        for i in range(k - 1, -1, -1):
            alpha[i] = self.rho[i] * float(delta @ B[:, i])          # rho_i s_i . q
            delta[k + i] -= alpha[i]                                 # q -= alpha_i y_i
        yy = float(B[2 * k - 1, 2 * k - 1])
        delta *= (1.0 / self.rho[-1]) / yy
        for i in range(k):
            beta = self.rho[i] * float(delta @ B[:, k + i])           # rho_i y_i . r
            delta[i] += alpha[i] - beta                              # r += (alpha_i - beta) s_i
        if g.is_cuda:
            from ..ops.native import lincomb
            q = lincomb(delta.tolist(), basis)     # one pass, no [2k + 1, D] stack
            if q is not None:
                return q
        V = torch.stack(basis)
        return delta.to(V.device, V.dtype) @ V


class LBFGS(Optimizer):
    def __init__(self, normalization=None, num_corrections: int = DEFAULT_NUM_CORRECTIONS,
                 tolerance: float = DEFAULT_TOLERANCE, max_iterations: int = DEFAULT_MAX_ITER,
                 constraints=None, track_state: bool = True):
        super().__init__(tolerance, max_iterations, normalization, constraints, track_state)
        self.m = num_corrections
        self.history = _History(num_corrections)
        self._failed_once = False
        self._finished = False
        self._inner_iter = 0
        # smooth (un-penalised) value/gradient at the current point, used for the history
        self._smooth_f = None
        self._smooth_g = None
        self._spec = None        # _Plan queued for the next iteration
        self.wasted_spec_passes = 0   # speculative margin passes queued but never used (diagnostics)
        self.plans_used = 0           # iterations run from a deep plan (diagnostics)
        self.plans_rejected = 0       # deep plans whose step the line search did not accept at t = 1

    def drop_speculation(self):
        """Forget the work queued for the next iteration (its direction and margin pass): that iteration then
        computes both itself. Benchmarks call this between untimed and timed iterations, so no timed iteration's
        work runs before the timer starts."""
        self._abandon(self._spec)
        self._spec = None

    def _abandon(self, plan: Optional[_Plan]):
        """Drop a queued plan. A deep plan's speculative passes moved the data backend's margin state forward:
        it is restored (unless other passes have run on that data since, which then own the state)."""
        if plan is None:
            return
        if plan.deep or plan.mls is not None:
            self.wasted_spec_passes += 1
        if plan.deep and plan.data is not None and plan.passes == self._pass_count(plan.data):
            plan.data.ls_restore(plan.ck_start)

    def is_done(self) -> bool:
        done = super().is_done()
        if done and self._spec is not None:
            # no further iteration: leave the data at the last ACCEPTED point (its cached margins are read next)
            self._abandon(self._spec)
            self._spec = None
        return done

    def _margin_speculation_pays(self, state: OptimizerState) -> bool:
        """Whether to queue the next iteration's margin pass during the history push. The pass is wasted when the
        iteration then stops on the loss tolerance (short warm-started GAME updates often do), so it is queued only
        while the last loss drop is well above that tolerance (the drop shrinks geometrically near convergence)."""
        if self.loss_abs_tol <= 0.0 or self.previous is None:
            return True
        try:
            drop = float(self.previous.loss) - float(state.loss)
        except (TypeError, ValueError):
            return True
        return drop > SPECULATE_LOSS_MARGIN * self.loss_abs_tol

    def clear_inner_state(self):
        super().clear_inner_state()
        self._abandon(self._spec)
        self.history.clear()
        self._failed_once = False
        self._finished = False
        self._inner_iter = 0
        self._spec = None

    def _inner_state(self) -> dict:
        h = self.history
        return {"s": list(h.s), "y": list(h.y), "rho": list(h.rho),
                "gamma": None if h.gamma_t is None else float(h.gamma_t), "failed_once": self._failed_once,
                "finished": self._finished, "inner_iter": self._inner_iter, "smooth_f": self._smooth_f,
                "smooth_g": self._smooth_g}

    def _load_inner_state(self, d: dict):
        self.history.s, self.history.y, self.history.rho = list(d["s"]), list(d["y"]), list(d["rho"])
        h = self.history
        h.rho_t, h.gamma_t = [], None
        if h.s and _device_loop(h.s[0]) and d.get("gamma") is not None:
            dev = h.s[0].device      # device scalars of the sync-free two-loop (1/sy is exact-rounded either way)
            h.rho_t = [torch.tensor(r, dtype=torch.float64, device=dev) for r in h.rho]
            h.gamma_t = torch.tensor(d["gamma"], dtype=torch.float64, device=dev)
        self._failed_once, self._finished, self._inner_iter = d["failed_once"], d["finished"], d["inner_iter"]
        self._smooth_f, self._smooth_g = d["smooth_f"], d["smooth_g"]

    # -- L1 hooks (identity for plain L-BFGS) --------------------------------
    def _adjust(self, x, f, g):
        return f, g

    def _init(self, objective, data, state: OptimizerState):
        self._smooth_f, self._smooth_g = state.loss, state.gradient
        adj_f, adj_g = self._adjust(state.coefficients, state.loss, state.gradient)
        state.loss, state.gradient = adj_f, adj_g

    def _direction(self, state: OptimizerState) -> torch.Tensor:
        return self.history.apply_inverse(state.gradient, negate=True)

    def _prefetch(self, state: OptimizerState, d: torch.Tensor):
        """Replicated device vectors: the device vector (g.d, d.d, x0.x0, x0.d), fetched later in ONE host
        synchronisation (the descent test, the first trial step 1/||d||, the zero-direction test and the L2 terms
        of the margin line search would otherwise each synchronise); None elsewhere."""
        if not _device_loop(d):
            return None
        return self._prefetch_of(state.coefficients, state.gradient, d)

    @staticmethod
    def _prefetch_of(x0: torch.Tensor, g: torch.Tensor, d: torch.Tensor) -> torch.Tensor:
        if NATIVE_PAIR:
            from ..ops.native import ls_dots
            out = ls_dots(x0, g, d)              # one launch instead of four dot products and a stack
            if out is not None:
                return out
        return torch.stack([torch.dot(g, d), torch.dot(d, d), torch.dot(x0, x0), torch.dot(x0, d)])

    @staticmethod
    def _pass_count(data):
        n = (getattr(data, "n_fwd", None), getattr(data, "n_t", None))
        return None if n[0] is None else n

    def _speculate_margins(self, objective, data, x, d):
        """The next iteration's margin line search (direction pass queued now, t0 = 1), or None."""
        if (not SPECULATE_MARGINS or not MARGIN_LINE_SEARCH or self.constraints
                or not hasattr(objective, "margin_line_search") or self._pass_count(data) is None):
            return None
        from ..function.objective import DEFERRED_DOTS
        mls = objective.margin_line_search(data, x, d, 1.0, dots=DEFERRED_DOTS)
        return None if mls is None else (mls, self._pass_count(data))

    def _queue_plan(self, objective, data, x, g, h: "_History", with_mls: bool, allow_inplace: bool) -> _Plan:
        """Queue the iteration that starts at (x, g) with history ``h``: its direction and line-search dots, and
        (``with_mls``) its margin pass -- as a DEEP plan (also the gradient at t = 1, the history pair and one
        readback; the pass writes the backend's other margin buffer pair) where the backend supports it, else
        in place (only when ``allow_inplace``: the current step is already accepted)."""
        dn = h.apply_inverse(g, negate=True)
        deep = (PLAN and with_mls and SPECULATE_MARGINS and MARGIN_LINE_SEARCH
                and callable(getattr(data, "ls_checkpoint", None)) and callable(getattr(data, "ls_finish_fused", None))
                and hasattr(objective, "margin_line_search")
                and getattr(objective.normalization, "factors", None) is None
                and getattr(objective.normalization, "shifts", None) is None
                and self._pass_count(data) is not None and dn.is_contiguous() and x.is_contiguous())
        if deep:
            from ..function.objective import DEFERRED_DOTS
            from ..ops.native import lbfgs_pair, ls_dots
            pack = torch.empty(16, dtype=torch.float64, device=g.device)
            pre = ls_dots(x, g, dn, out=pack[0:4])
            if pre is not None:
                plan = _Plan(x, g, dn, pre)
                plan.ck_start = data.ls_checkpoint()
                mls = objective.margin_line_search(data, x, dn, 1.0, dots=DEFERRED_DOTS,
                                                   ls_opts={"alt": True, "stats_out": pack[4:6]})
                if mls is not None:
                    plan.ck_fwd = data.ls_checkpoint()
                    host = _pinned_slot(g.device)
                    host[:6].copy_(pack[:6], non_blocking=True)          # readback A: pre + first trial
                    ev_a = torch.cuda.Event()
                    ev_a.record()
                    x1, _, g1 = data.ls_finish_fused(objective.loss, 1.0, x, dn, objective.l2_weight)
                    objective.n_value_grad += 1
                    r = lbfgs_pair(x1, x, g1, g, out=pack[6:11])
                    if r is not None:
                        plan.deep, plan.mls, plan.data = True, mls, data
                        plan.x1, plan.g1 = x1, g1
                        plan.s, plan.y, plan.out = r
                        plan.ck_fin = data.ls_checkpoint()
                        plan.passes = self._pass_count(data)
                        plan.host, plan.ev_a = host, ev_a
                        plan.host[6:11].copy_(pack[6:11], non_blocking=True)   # readback B: pair scalars
                        plan.ev = torch.cuda.Event()
                        plan.ev.record()
                        return plan
                    data.ls_restore(plan.ck_fwd)
                    plan.mls = (mls, self._pass_count(data))
                    return plan
                if allow_inplace:
                    plan.mls = self._speculate_margins(objective, data, x, dn)
                return plan
        return _Plan(x, g, dn, self._prefetch_of(x, g, dn),
                     self._speculate_margins(objective, data, x, dn) if with_mls and allow_inplace else None)

    def _search(self, objective, data, state: OptimizerState, d: torch.Tensor, pre=None, spec_mls=None):
        """``pre``: host list or device vector from :meth:`_prefetch`. A device vector is read AFTER the margin
        line search has queued its direction pass (iterations > 0: t0 = 1 is known), so the GPU runs that pass
        while the host waits instead of idling through the synchronisation. ``spec_mls``: that search, already
        started during the previous iteration's history push (used only if no pass ran since)."""
        x0 = state.coefficients
        from ..utils.timing import trace_range
        use_mls = MARGIN_LINE_SEARCH and not self.constraints and hasattr(objective, "margin_line_search")
        if pre is not None and not isinstance(pre, list) and (self._inner_iter == 0 or not use_mls):
            pre = pre.tolist()
        mls = None
        if use_mls:
            t0 = (1.0 / pre[1] ** 0.5 if pre is not None else 1.0 / _norm(d)) if self._inner_iter == 0 else 1.0
            lazy = pre is not None and not isinstance(pre, list)
            # a device ``pre`` is read after the direction pass is queued: the L2 dots are assigned then, not
            # recomputed (vdots would cost three reductions and a host synchronisation of their own)
            from ..function.objective import DEFERRED_DOTS
            if (spec_mls is not None and pre is not None and t0 == 1.0 and spec_mls[0].x0 is x0
                    and spec_mls[0].d is d and spec_mls[1] == self._pass_count(data)):
                mls = spec_mls[0]
            else:
                mls = objective.margin_line_search(data, x0, d, t0, dots=None if pre is None else
                                                   (DEFERRED_DOTS if lazy else (pre[2], pre[3], pre[1])))
            if (lazy and mls is not None and t0 == 1.0 and GATED_FINISH and callable(getattr(data, "ls_finish_gated", None))
                    and callable(getattr(data, "ls_finish_fused", None))
                    and mls.x0 is x0 and mls.d is d and getattr(objective.normalization, "factors", None) is None
                    and getattr(objective.normalization, "shifts", None) is None and data.ls_gate_supported()):
                got = self._gated_first_trial(objective, data, state, mls, pre)
                if got is not None:
                    return got
                pre = self._gated_pre
            elif lazy:
                pre = pre.tolist()
            if mls is not None and mls.l2 > 0 and pre is not None:
                mls.a, mls.b, mls.c = pre[2], pre[3], pre[1]
        with trace_range("line-search setup"):
            if pre is not None:
                g0 = pre[0]
                t0 = 1.0 / pre[1] ** 0.5 if self._inner_iter == 0 else 1.0
                if not pre[1] > 0 and not vector_space.current().any_nonzero(d):
                    raise _ZeroDirection()
            else:
                g0 = _dot(state.gradient, d)
                t0 = 1.0 / _norm(d) if self._inner_iter == 0 else 1.0
        if mls is not None:
            # trials in margin space (one elementwise pass each), full gradient only at the accepted step
            _, _, _, t = strong_wolfe(lambda tt: (*mls.eval(tt), tt), state.loss, g0, t0)  # payload = the step
            return mls.finish(t)

        def phi(t):
            x = x0 + t * d
            f, g = objective.calculate(data, x)
            return f, _dot(g, d), (x, f, g)

        t, _, _, (x, f, g) = strong_wolfe(phi, state.loss, g0, t0)
        return x, f, g

    def _gated_first_trial(self, objective, data, state: OptimizerState, mls, pre_dev: torch.Tensor):
        """The gated finish (GATED_FINISH): returns (x, f, g) of the accepted t = 1, or None after restoring the
        data's line-search state (the search then continues from its first trial; ``self._gated_pre`` holds the
        host copy of ``pre``)."""
        from ..function.objective import DEFERRED_DOTS  # noqa: F401  (mls built with deferred dots)
        from .line_search import strong_wolfe as _sw
        ck = data.ls_checkpoint()
        c1, c2 = 1e-4, 0.9
        vals, x1, F1, g1 = data.ls_finish_gated(objective.loss, pre_dev, state.loss, mls.l2, c1, c2, mls.x0, mls.d)
        pre, F, D, dev_acc = vals[0:4], vals[4], vals[5], vals[6] == 1.0
        self._gated_pre = pre
        if mls.l2 > 0:
            mls.a, mls.b, mls.c = pre[2], pre[3], pre[1]

        def first_trial_only(t):
            if t != 1.0:
                raise _Unplanned()
            return (*mls.adjust(F, D, 1.0), None)

        host_acc = False
        if pre[1] > 0 and pre[0] < 0:
            try:
                t, _, _, _ = _sw(first_trial_only, state.loss, pre[0], 1.0, c1, c2)
                host_acc = t == 1.0
            except (_Unplanned, LineSearchFailed):
                host_acc = False
        self.gated_seen = getattr(self, "gated_seen", 0) + 1
        if host_acc and dev_acc and not GATED_TEST_DISAGREE:
            self.gated_used = getattr(self, "gated_used", 0) + 1
            objective.n_value_grad += 1
            f = F1
            if mls.l2 > 0:
                f = f + 0.5 * mls.l2 * (mls.a + 2.0 * 1.0 * mls.b + 1.0 * 1.0 * mls.c)
            return x1, f, g1
        data.ls_restore(ck, t0_host=(F, D))
        return None

    def _run_one_iteration(self, objective, data, state: OptimizerState) -> OptimizerState:
        if self._finished:
            return state
        spec, self._spec = self._spec, None
        use = spec is not None and spec.x is state.coefficients and spec.g is state.gradient
        if use and spec.deep and not (spec.data is data and spec.passes == self._pass_count(data)):
            use = False
        if spec is not None and not use:
            self._abandon(spec)
            spec = None
        if spec is not None and spec.deep:
            return self._run_planned(objective, data, state, spec)
        return self._run_unplanned(objective, data, state, spec)

    def _run_planned(self, objective, data, state: OptimizerState, p: _Plan) -> OptimizerState:
        """One iteration from a deep plan: read its line-search scalars (readback A; the GPU meanwhile runs the
        speculative gradient pass), take the line search's decision on them; if t = 1 stands, queue the NEXT plan
        (as if the pair passes), then read the pair's scalars (readback B) and commit, else fall back to the
        ordinary search."""
        from ..utils.timing import trace_range
        with trace_range("plan readback A"):
            p.ev_a.synchronize()
            vals = p.host[:6].tolist()
        pre, F, D = vals[0:4], vals[4], vals[5]
        mls = p.mls
        if mls.l2 > 0:
            mls.a, mls.b, mls.c = pre[2], pre[3], pre[1]

        def first_trial_only(t):
            if t != 1.0:
                raise _Unplanned()
            return (*mls.adjust(F, D, 1.0), None)

        accepted = None
        self._plans_seen = getattr(self, "_plans_seen", 0) + 1
        pre_real = pre
        if PLAN_TEST_REJECT and self._plans_seen % PLAN_TEST_REJECT == 0:
            pre = pre[:1] + [0.0] + pre[2:]           # forced fallback (the search itself uses the real values)
        if pre[1] > 0 and pre[0] < 0:
            try:
                t, f, _, _ = strong_wolfe(first_trial_only, state.loss, pre[0], 1.0)
                accepted = f if t == 1.0 else None
            except (_Unplanned, LineSearchFailed):
                accepted = None
        if accepted is None:
            # the ordinary search from this plan's direction pass (the margins at x and X d are intact)
            self.plans_rejected += 1
            data.ls_restore(p.ck_fwd, t0_host=(F, D))
            return self._run_unplanned(objective, data, state,
                                       _Plan(p.x, p.g, p.d, pre_real, (mls, self._pass_count(data))))
        nxt = None
        with trace_range("plan of the next iteration"):
            if state.iter + 2 <= self.max_iterations and len(self.history.rho_t) == len(self.history.s):
                h = self.history._with_pair(p.s, p.y, p.out[2], p.out[3])
                nxt = self._queue_plan(objective, data, p.x1, p.g1, h, self._margin_speculation_pays(state),
                                       allow_inplace=False)
        with trace_range("plan readback B"):
            p.ev.synchronize()
            vals = p.host[6:11].tolist()
        sy, gg = vals[0], vals[4]
        self.plans_used += 1
        if not (sy > 1e-300) or sy != sy:
            # the step stands, the pair does not: the next plan assumed it
            self._abandon(nxt)
            nxt = None
            data.ls_restore(p.ck_fin)
        else:
            self.history.commit(p.s, p.y, sy, p.out[2], p.out[3])
        self._spec = nxt
        self._failed_once = False
        self._smooth_f, self._smooth_g = accepted, p.g1
        self._inner_iter += 1
        new = OptimizerState(p.x1, accepted, p.g1, state.iter + 1)
        new._grad_norm = gg ** 0.5
        return new

    def _run_unplanned(self, objective, data, state: OptimizerState, spec: Optional[_Plan] = None) -> OptimizerState:
        from ..utils.timing import trace_range
        try:
            with trace_range("two-loop direction"):
                spec_mls = None
                if spec is not None:
                    d, pre, spec_mls = spec.d, spec.pre, spec.mls   # queued during the last history push
                else:
                    d = self._direction(state)
                    pre = self._prefetch(state, d)
                # device: d.d > 0 decides later, in _search (d.d == 0 -- all zero or underflow -- checks exactly)
                nonzero = pre is not None or vector_space.current().any_nonzero(d)
            if not nonzero:
                self._finished = True  # zero (pseudo-)gradient: stationary point
                return state
            x, f, g = self._search(objective, data, state, d, pre, spec_mls)
        except _ZeroDirection:
            self._finished = True
            return state
        except LineSearchFailed:
            if not self._failed_once and len(self.history.s) > 0:
                self._failed_once = True
                self.history.clear()
                return self._run_one_iteration(objective, data, state)
            self._finished = True
            return state
        self._failed_once = False
        with trace_range("history push"):
            # a device-scalar loss (margin line search) is read in the pair's synchronisation
            f_dev = f if isinstance(f, torch.Tensor) else None
            spec_fn = None
            if (SPECULATE_DIRECTION and type(self)._direction is LBFGS._direction and not self.constraints
                    and _device_loop(g) and g.numel() < GRAM_MIN_DIM and not vector_space.current().sharded
                    and state.iter + 2 <= self.max_iterations):         # the next iteration can run
                # plain L-BFGS: the next state is (x, g) as is (no L1 adjustment, no box projection)
                with_mls = self._margin_speculation_pays(state)
                spec_fn = lambda h: self._queue_plan(objective, data, x, g, h, with_mls, allow_inplace=True)
            pushed, gg, f_host, nxt = self.history.push_pair(x, state.coefficients, g, self._smooth_g, extra=f_dev,
                                                             speculate=spec_fn)
            if f_dev is not None:
                f = f_host
            if nxt is not None and not pushed:
                self._abandon(nxt)
                nxt = None
            self._spec = nxt
        self._smooth_f, self._smooth_g = f, g
        self._inner_iter += 1
        adj_f, adj_g = self._adjust(x, f, g)
        x = project_box(x, self.constraints)
        new = OptimizerState(x, adj_f, adj_g, state.iter + 1)
        if gg is not None and adj_g is g:
            new._grad_norm = gg ** 0.5      # the convergence test needs no further synchronisation
        return new


class _ZeroDirection(Exception):
    """The search direction is exactly zero (stationary point)."""


class OWLQN(LBFGS):
    """Orthant-wise limited-memory quasi-Newton for L1 / elastic-net (L1 part in the optimizer)."""

    def __init__(self, l1_weight: float, normalization=None, num_corrections: int = DEFAULT_NUM_CORRECTIONS,
                 tolerance: float = DEFAULT_TOLERANCE, max_iterations: int = DEFAULT_MAX_ITER,
                 constraints=None, track_state: bool = True):
        super().__init__(normalization, num_corrections, tolerance, max_iterations, constraints, track_state)
        self.l1_weight = float(l1_weight)

    # pseudo-gradient (Andrew & Gao 2007)
    def _pseudo_gradient(self, x, g):
        lam = self.l1_weight
        at_zero = x == 0
        dplus = g + lam
        dminus = g - lam
        pg_zero = torch.where(dminus > 0, dminus, torch.where(dplus < 0, dplus, torch.zeros_like(g)))
        return torch.where(at_zero, pg_zero, g + lam * torch.sign(x))

    def _adjust(self, x, f, g):
        return f + self.l1_weight * vector_space.current().abs_sum(x), self._pseudo_gradient(x, g)

    def _direction(self, state):
        d = self.history.apply_inverse(state.gradient, negate=True)
        # keep only components that descend along the pseudo-gradient
        return torch.where(d * state.gradient < 0, d, torch.zeros_like(d))

    def _prefetch(self, state, d):
        return None        # the orthant-masked direction is tested for zero before the search, as before

    def _search(self, objective, data, state, d, pre=None, spec_mls=None):
        x0 = state.coefficients
        pg = state.gradient
        orthant = torch.where(x0 != 0, torch.sign(x0), torch.sign(-pg))
        # first trial as Breeze OWLQN.determineStepSize: 0.5 / ||adjusted gradient|| on iteration 0, else 1
        t0 = 0.5 / _norm(pg) if self._inner_iter == 0 else 1.0
        shrink = 0.1 if self._inner_iter < 1 else 0.5

        def phi(t):
            x = x0 + t * d
            x = torch.where(torch.sign(x) != orthant, torch.zeros_like(x), x)
            f, g = objective.calculate(data, x)
            adj_f, adj_g = self._adjust(x, f, g)
            return adj_f, _dot(adj_g, d), (x, f, g)

        g0 = _dot(pg, d)
        if g0 >= 0:
            raise LineSearchFailed("OWL-QN: not a descent direction")
        _, _, _, (x, f, g) = backtracking(phi, state.loss, g0, t0, shrink)
        return x, f, g
