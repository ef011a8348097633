"""Line searches used by L-BFGS (strong Wolfe) and OWL-QN (backtracking Armijo).

The reference delegates these to Breeze 0.11.2 (``breeze.optimize.StrongWolfeLineSearch`` with
``maxZoomIter = 10, maxLineSearchIter = 10`` and ``BacktrackingLineSearch``); Breeze is external, so this is a
fresh implementation of the textbook algorithms (Nocedal & Wright, Alg. 3.5/3.6 with cubic interpolation),
targeting model-quality parity rather than bitwise iterates.

``phi(t)`` returns ``(value, directional_derivative, payload)``; the payload (new point, gradient, ...) of the
accepted step is returned so the caller never re-evaluates the objective.
"""
from __future__ import annotations

import math


EXTRAPOLATION = 1.5     # strong Wolfe: the next trial after a short one is t * EXTRAPOLATION


class LineSearchFailed(RuntimeError):
    pass


def _cubic_min(a, fa, ga, b, fb, gb):
    """Minimiser of the cubic interpolating (a,fa,ga),(b,fb,gb); falls back to bisection."""
    d1 = ga + gb - 3.0 * (fa - fb) / (a - b)
    disc = d1 * d1 - ga * gb
    if disc < 0 or not math.isfinite(disc):
        return 0.5 * (a + b)
    d2 = math.copysign(math.sqrt(disc), b - a)
    denom = gb - ga + 2.0 * d2
    if denom == 0 or not math.isfinite(denom):
        return 0.5 * (a + b)
    t = b - (b - a) * (gb + d2 - d1) / denom
    lo, hi = min(a, b), max(a, b)
    # safeguard: keep away from the bracket ends
    span = hi - lo
    if not math.isfinite(t) or t <= lo + 0.1 * span or t >= hi - 0.1 * span:
        return 0.5 * (a + b)
    return t


def strong_wolfe(phi, f0: float, g0: float, t_init: float = 1.0, c1: float = 1e-4, c2: float = 0.9,
                 max_iter: int = 10, max_zoom: int = 10):
    """Return ``(t, f, g, payload)`` satisfying the strong Wolfe conditions (best effort)."""
    if g0 >= 0:
        raise LineSearchFailed(f"not a descent direction (g0={g0})")
    t_prev, f_prev, g_prev, p_prev = 0.0, f0, g0, None
    t = t_init
    best = None

    def zoom(lo, flo, glo, plo, hi, fhi, ghi, phi_hi):
        nonlocal best
        for _ in range(max_zoom):
            tj = _cubic_min(lo, flo, glo, hi, fhi, ghi)
            fj, gj, pj = phi(tj)
            if fj > f0 + c1 * tj * g0 or fj >= flo:
                hi, fhi, ghi = tj, fj, gj
            else:
                if abs(gj) <= -c2 * g0:
                    return tj, fj, gj, pj
                if gj * (hi - lo) >= 0:
                    hi, fhi, ghi = lo, flo, glo
                lo, flo, glo, plo = tj, fj, gj, pj
        # zoom exhausted: accept the best sufficient-decrease point if any
        if plo is not None and flo < f0:
            return lo, flo, glo, plo
        raise LineSearchFailed("zoom did not converge")

    for i in range(max_iter):
        ft, gt, pt = phi(t)
        if not math.isfinite(ft):
            # step too long: shrink and retry
            t = 0.5 * (t_prev + t)
            continue
        if ft > f0 + c1 * t * g0 or (i > 0 and ft >= f_prev):
            return zoom(t_prev, f_prev, g_prev, p_prev, t, ft, gt, pt)
        if abs(gt) <= -c2 * g0:
            return t, ft, gt, pt
        if gt >= 0:
            return zoom(t, ft, gt, pt, t_prev, f_prev, g_prev, p_prev)
        t_prev, f_prev, g_prev, p_prev = t, ft, gt, pt
        t = t * EXTRAPOLATION
    if p_prev is not None and f_prev < f0:
        return t_prev, f_prev, g_prev, p_prev
    raise LineSearchFailed("line search exceeded max iterations")


def backtracking(phi, f0: float, g0: float, t_init: float = 1.0, shrink: float = 0.5, c1: float = 1e-4,
                 max_iter: int = 30):
    """Armijo backtracking; ``phi`` as in :func:`strong_wolfe`."""
    t = t_init
    for _ in range(max_iter):
        ft, gt, pt = phi(t)
        if math.isfinite(ft) and ft <= f0 + c1 * t * g0:
            return t, ft, gt, pt
        t *= shrink
    raise LineSearchFailed("backtracking exceeded max iterations")
