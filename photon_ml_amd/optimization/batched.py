"""Batched per-entity GLM solvers for random effects.

The reference solves one small ``SingleNodeOptimizationProblem`` per entity inside ``RDD.mapValues``
(``photon-api/.../algorithm/RandomEffectCoordinate.scala:108-119``,
``optimization/SingleNodeOptimizationProblem.scala:85-103``). Here all entities of a size BUCKET are solved
together as one batch of dense padded problems ``X [B, n, d]`` (padding rows carry weight 0, padding columns are
all-zero so their coefficients stay 0): every optimizer step is a handful of batched GEMV/GEMMs (``bmm``,
rocBLAS/hipBLASLt on MI355X — plain library GEMMs) plus elementwise masks, so tens of thousands of tiny solves
become a few large device launches.

Per entity the semantics of the scalar optimizers are kept: Photon's convergence rules (tolerances from the
state at zero, MaxIterations / ObjectiveNotImproving / FunctionValuesConverged / GradientConverged), TRON's
trust-region constants and truncated CG, L-BFGS two-loop with m = 10 history, OWL-QN pseudo-gradient and orthant
projection. Entities converge independently (masked); the batch loop ends when every entity is done.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Optional

import torch

from .optimizer import ConvergenceReason

REASON_CODES = {0: None, 1: ConvergenceReason.MAX_ITERATIONS, 2: ConvergenceReason.OBJECTIVE_NOT_IMPROVING,
                3: ConvergenceReason.FUNCTION_VALUES_CONVERGED, 4: ConvergenceReason.GRADIENT_CONVERGED}


class BatchedGLMData:
    """Dense padded batch of per-entity GLM problems. Vectors are ``[B, d]``."""

    def __init__(self, X: torch.Tensor, y: torch.Tensor, offsets: torch.Tensor, weights: torch.Tensor):
        self.X = X  # [B, n, d]
        self.y = y  # [B, n]
        self.o = offsets
        self.w = weights  # 0 on padding rows
        self._dzz_key = None
        self._dzz = None

    # ---- batch vector space: per-entity dot products / broadcasting of per-entity scalars
    @property
    def n_batch(self) -> int:
        return self.X.shape[0]

    def _regular_ptr(self):
        p = getattr(self, "_ptr", None)
        if p is None:
            B, _, d = self.X.shape
            p = self._ptr = torch.arange(B + 1, dtype=torch.int64, device=self.X.device) * d
        return p

    def bdot(self, a, b):
        if a.is_cuda and a.dtype == torch.float64 and a.is_contiguous() and b.is_contiguous():
            from ..ops.native import segdot   # one deterministic kernel instead of multiply + reduce
            return segdot(a.view(-1), b.view(-1), self._regular_ptr(), 0)
        return (a * b).sum(-1)

    def bexp(self, s):
        return s.unsqueeze(-1)

    def cg_step(self, step, r, d, Hd, rtr, on, delta, l2: float = 0.0):
        """Fused truncated-CG iteration for every problem (``seg_cg_step`` over the regular [B, d] layout)."""
        from ..ops.native import seg_cg_step
        seg_cg_step(self._regular_ptr(), step.view(-1), r.view(-1), d.view(-1), Hd.contiguous().view(-1), rtr, on,
                    delta, l2)

    def babs_sum(self, a):
        return a.abs().sum(-1)

    @property
    def shape(self):
        return tuple(self.X.shape)

    def _mv(self, v, trans: bool = False):
        from ..ops.native import batched_gemv
        if self.X.shape[1] == self.X.shape[2] and self.X.dtype == torch.float64:
            return batched_gemv(self.X, v, trans)   # small square blocks (row-space problems): HIP kernel
        M = self.X.transpose(1, 2) if trans else self.X
        return torch.bmm(M, v.unsqueeze(-1)).squeeze(-1)

    def margins(self, W: torch.Tensor) -> torch.Tensor:
        return self._mv(W) + self.o

    def value_grad(self, loss, W, l2: float):
        z = self.margins(W)
        l, dl = loss.loss_and_dz(z, self.y)
        f = (self.w * l).sum(1)
        g = self._mv(self.w * dl, trans=True)
        if l2 > 0:
            f = f + 0.5 * l2 * (W * W).sum(1)
            g = g + l2 * W
        return f, g

    def _dzz_at(self, loss, W):
        # cache keyed by tensor identity + in-place version (holding the reference keeps W alive, so its
        # storage cannot be recycled under the key); no O(D) comparison / copy per Hessian-vector product
        key = self._dzz_key
        if key is not None and key[0] is W and key[1] == W._version and key[2] is loss:
            return self._dzz
        self._dzz = self.w * loss.dzz(self.margins(W), self.y)
        self._dzz_key = (W, W._version, loss)
        return self._dzz

    def hv(self, loss, W, V, l2: float):
        D = self._dzz_at(loss, W)
        if self.X.shape[1] == self.X.shape[2] and self.X.dtype == torch.float64:
            from ..ops.native import batched_hv
            return batched_hv(self.X, D, V, l2)
        xv = torch.bmm(self.X, V.unsqueeze(-1)).squeeze(-1)
        h = torch.bmm(self.X.transpose(1, 2), (D * xv).unsqueeze(-1)).squeeze(-1)
        return h + l2 * V if l2 > 0 else h

    def hdiag(self, loss, W, l2: float):
        D = self.w * loss.dzz(self.margins(W), self.y)
        h = torch.bmm((self.X * self.X).transpose(1, 2), D.unsqueeze(-1)).squeeze(-1)
        return h + l2 if l2 > 0 else h


class SegmentedGLMData:
    """All entities of a random-effect coordinate as ONE block-diagonal sparse GLM.

    Rows are the active rows sorted by entity; entity ``e`` owns the contiguous coefficient range
    ``[col_ptr[e], col_ptr[e+1])`` (its INDEX_MAP-projected features), so the design matrix is block diagonal and
    a "batched" solve is a single vector of length ``D_total = sum d_e`` with per-entity scalars obtained by
    segment sums. The matrix products run on the GLM HIP kernels (``matvec`` = forward pass, ``rmatvec`` =
    transpose pass over column tiles / windows) — no padding, any mix of entity sizes, one launch sequence for all
    entities (reference ``SingleNodeOptimizationProblem`` per entity).
    """

    def __init__(self, glm, row_entity: torch.Tensor, col_entity: torch.Tensor, n_entities: int, y: torch.Tensor,
                 weights: torch.Tensor, offsets: torch.Tensor):
        self.glm = glm
        self.row_entity = row_entity  # sorted: rows grouped by entity
        self.col_entity = col_entity  # sorted: each entity's coefficients are contiguous
        self.B = int(n_entities)
        self.y, self.w, self.o = y, weights, offsets
        dev = y.device
        ar = torch.arange(self.B + 1, device=dev)
        self.row_ptr = torch.searchsorted(row_entity, ar).to(torch.int64)
        self.col_ptr = torch.searchsorted(col_entity, ar).to(torch.int64)
        self._dzz_key = None
        self._dzz = None

    @property
    def n_batch(self) -> int:
        return self.B

    # per-entity reductions over contiguous segments: deterministic segmented kernel (no scatter atomics)
    def bdot(self, a, b):
        from ..ops.native import segdot
        return segdot(a, b, self.col_ptr, 0)

    def bexp(self, s):
        from ..ops.native import seg_expand
        return seg_expand(s, self.col_ptr, self.col_entity.numel())

    def babs_sum(self, a):
        from ..ops.native import segdot
        return segdot(a, None, self.col_ptr, 2)

    def _rowsum(self, v):
        from ..ops.native import segdot
        return segdot(v, None, self.row_ptr, 1)

    def cg_step(self, step, r, d, Hd, rtr, on, delta, l2: float = 0.0):
        """Fused truncated-CG iteration over all entity segments (see ``ops.native.seg_cg_step``); ``Hd``
        without the L2 term (added in the kernel)."""
        from ..ops.native import seg_cg_step
        seg_cg_step(self.col_ptr, step, r, d, Hd, rtr, on, delta, l2)

    supports_active = True

    def _set_active(self, active):
        """Entity-masked GLM passes (``DeviceGLMData.set_entity_mask``): blocks / tiles of entities outside
        ``active`` are skipped; their margins and gradient entries are not computed (the callers only read the
        active entities)."""
        glm = self.glm
        if not MASKED_PASSES or not hasattr(glm, "entity_mask_geometry"):
            return
        if active is None:
            if getattr(self, "_active_key", None) is not None:
                glm.set_entity_mask(None)
                self._active_key = None
            return
        geo = glm.entity_mask_geometry(self.row_entity, self.col_entity)
        if not geo:
            return
        glm.set_entity_mask(active, geo)           # a few device ops, no host synchronisation
        self._active_key = True

    def margins(self, W, active=None):
        self._set_active(active)
        return self.glm.matvec(W) + self.o

    def value_grad(self, loss, W, l2: float, active=None):
        z = self.margins(W, active)
        l, dl = loss.loss_and_dz(z, self.y)
        f = self._rowsum(self.w * l)
        g = self.glm.rmatvec(self.w * dl)
        if l2 > 0:
            f = f + 0.5 * l2 * self.bdot(W, W)
            g = g + l2 * W
        return f, g

    def _dzz_at(self, loss, W):
        # cache keyed by tensor identity + in-place version (holding the reference keeps W alive, so its
        # storage cannot be recycled under the key); no O(D) comparison / copy per Hessian-vector product
        key = self._dzz_key
        mk = getattr(self, "_active_key", None)
        # a cache filled under an entity mask covers that mask's entities; inside batched_tron every later mask
        # at the same W is a subset (CG masks shrink, rejected steps keep W, the active set only shrinks)
        if (key is not None and key[0] is W and key[1] == W._version and key[2] is loss
                and (key[3] is None or mk is not None)):
            return self._dzz
        self._dzz = self.w * loss.dzz(self.glm.matvec(W) + self.o, self.y)
        self._dzz_key = (W, W._version, loss, None if mk is None else True)
        return self._dzz

    def hv(self, loss, W, V, l2: float, active=None):
        self._set_active(active)
        D = self._dzz_at(loss, W)
        h = self.glm.rmatvec(D * self.glm.matvec(V))
        return h + l2 * V if l2 > 0 else h

    def hdiag(self, loss, W, l2: float):
        D = self.w * loss.dzz(self.margins(W), self.y)
        h = self.glm.rmatvec(D, square=True)
        return h + l2 if l2 > 0 else h


def _bn(data, a):
    return torch.sqrt(data.bdot(a, a).clamp(min=0))


@dataclass
class BatchedResult:
    W: torch.Tensor          # [B, d] (dense batch) or [D_total] (segmented) coefficients
    f: torch.Tensor          # [B] final objective (incl. regularisation)
    iters: torch.Tensor      # [B] iterations
    reason: torch.Tensor     # [B] int convergence codes (see REASON_CODES)


class _Convergence:
    """Vectorised Photon convergence bookkeeping."""

    def __init__(self, data, f0z, g0z, tol, max_iter, device):
        self.data = data
        self.loss_tol = f0z * tol
        self.grad_tol = _bn(data, g0z) * tol
        self.max_iter = max_iter

    def check(self, it, f_new, f_prev, g_new, completed, not_improving):
        """Return reason codes (0 = continue) for entities whose iteration just completed."""
        reason = torch.zeros_like(it)
        r_max = it >= self.max_iter
        r_fv = (f_new - f_prev).abs() <= self.loss_tol
        r_gc = _bn(self.data, g_new) <= self.grad_tol
        reason = torch.where(completed & r_gc, torch.full_like(reason, 4), reason)
        reason = torch.where(completed & r_fv, torch.full_like(reason, 3), reason)
        reason = torch.where(not_improving, torch.full_like(reason, 2), reason)
        reason = torch.where((completed | not_improving) & r_max, torch.full_like(reason, 1), reason)
        return reason


# block-diagonal passes skip the row blocks / column tiles of entities that stopped iterating (PML_RE_MASKED=0: off)
MASKED_PASSES = os.environ.get("PML_RE_MASKED", "1") != "0"

# PML_TRON_STATS=1: record, per CG step of the block-diagonal TRON, the fraction of rows whose entity is still
# iterating (how much of each Hessian-vector pass is wasted on converged entities); read by bench_game.py
_TRON_STATS = [] if os.environ.get("PML_TRON_STATS") == "1" else None


def tron_stats():
    return _TRON_STATS


def batched_tron(data, loss, l2: float, W0: torch.Tensor, tol: float = 1e-5, max_iter: int = 15,
                 max_fail: int = 5, max_cg: int = 20, fused: Optional[bool] = None,
                 frozen: Optional[torch.Tensor] = None) -> BatchedResult:
    """Vectorised TRON (``photon-lib/.../optimization/TRON.scala:80-340``) over a batch of entities.

    ``frozen`` [B] bool: entities solved elsewhere (e.g. in their row space, ``row_space.py``) — kept at W0, not
    iterated, reason code 0.

    ``fused``: run each CG iteration's vector algebra as one segmented kernel (``data.cg_step``; default when the
    data provides it, i.e. the block-diagonal layout) instead of ~30 elementwise / reduction ops."""
    try:
        return _batched_tron(data, loss, l2, W0, tol, max_iter, max_fail, max_cg, fused, frozen)
    finally:
        if getattr(data, "supports_active", False):
            data._set_active(None)          # later users of the GLM data get full passes


def _batched_tron(data, loss, l2, W0, tol, max_iter, max_fail, max_cg, fused, frozen) -> BatchedResult:
    if fused is None:
        fused = hasattr(data, "cg_step") and os.environ.get("PML_FUSED_CG", "1") != "0"
    eta0, eta1, eta2 = 1e-4, 0.25, 0.75
    s1, s2, s3 = 0.25, 0.5, 4.0
    W = W0.clone()
    B = data.n_batch
    E = data.bexp
    dev = W.device
    f, g = data.value_grad(loss, W, l2)
    if bool((W0 == 0).all()):
        f0z, g0z = f, g
    else:
        f0z, g0z = data.value_grad(loss, torch.zeros_like(W), l2)
    conv = _Convergence(data, f0z, g0z, tol, max_iter, dev)
    delta = _bn(data, g)
    it = torch.zeros(B, dtype=torch.long, device=dev)
    fails = torch.zeros(B, dtype=torch.long, device=dev)
    reason = torch.zeros(B, dtype=torch.long, device=dev)
    # entities with an all-zero problem (no data) converge immediately
    active = torch.ones(B, dtype=torch.bool, device=dev)
    zero_g = _bn(data, g) == 0
    reason = torch.where(zero_g, torch.full_like(reason, 4), reason)
    active &= ~zero_g
    if frozen is not None:
        active &= ~frozen
        reason = torch.where(frozen, torch.zeros_like(reason), reason)
    guard = 0
    while bool(active.any()):
        guard += 1
        if guard > max_iter * (max_fail + 1) + 5:
            break
        # ---- truncated CG (masked per entity)
        step = torch.zeros_like(W)
        r = -g.clone()
        d = r.clone()
        rtr = data.bdot(r, r)
        cg_tol = 0.1 * _bn(data, g)
        cg_on = active.clone()
        if fused:
            rtr, delta = rtr.contiguous(), delta.to(torch.float64).contiguous()
        for _ in range(max_cg):
            cg_on &= torch.sqrt(rtr.clamp(min=0)) > cg_tol
            if not bool(cg_on.any()):
                break
            if _TRON_STATS is not None and hasattr(data, "row_ptr"):
                n_rows = (data.row_ptr[1:] - data.row_ptr[:-1]).to(torch.float64)
                _TRON_STATS.append(float((n_rows * cg_on).sum() / n_rows.sum().clamp(min=1)))
            act_kw = {"active": cg_on} if getattr(data, "supports_active", False) else {}
            if fused:
                Hd = data.hv(loss, W, d, 0.0, **act_kw)
                on8 = cg_on.to(torch.uint8)
                data.cg_step(step, r, d, Hd, rtr, on8, delta, l2)
                cg_on = on8.bool()
                continue
            Hd = data.hv(loss, W, d, l2, **act_kw)
            dHd = data.bdot(d, Hd)
            alpha = torch.where(cg_on, rtr / torch.where(dHd == 0, torch.ones_like(dHd), dHd),
                                torch.zeros_like(rtr))
            trial = step + E(alpha) * d
            hit = cg_on & (_bn(data, trial) > delta)
            # boundary solution for entities that leave the trust region
            std = data.bdot(step, d)
            sts = data.bdot(step, step)
            dtd = data.bdot(d, d)
            dsq = delta * delta
            rad = torch.sqrt((std * std + dtd * (dsq - sts)).clamp(min=0))
            tau = torch.where(std >= 0, (dsq - sts) / (std + rad).clamp(min=1e-300),
                              (rad - std) / dtd.clamp(min=1e-300))
            move = cg_on & ~hit
            step = torch.where(E(move), trial, step)
            step = torch.where(E(hit), step + E(tau) * d, step)
            r_new = torch.where(E(move), r - E(alpha) * Hd, r)
            r_new = torch.where(E(hit), r - E(tau) * Hd, r_new)
            rnew_tr = data.bdot(r_new, r_new)
            beta = torch.where(move, rnew_tr / torch.where(rtr == 0, torch.ones_like(rtr), rtr),
                               torch.zeros_like(rtr))
            d = torch.where(E(move), r_new + E(beta) * d, d)
            r = r_new
            rtr = torch.where(move, rnew_tr, rtr)
            cg_on &= ~hit
        # ---- trial step
        W_new = W + step
        gs = data.bdot(g, step)
        pred = -0.5 * (gs - data.bdot(step, r))
        f_new, g_new = data.value_grad(loss, W_new, l2, **({"active": active} if getattr(
            data, "supports_active", False) else {}))
        actual = f - f_new
        snorm = _bn(data, step)
        first = active & (it == 0)
        delta = torch.where(first, torch.minimum(delta, snorm), delta)
        den = f_new - f - gs
        alpha = torch.where(den <= 0, torch.full_like(den, s3),
                            torch.maximum(torch.full_like(den, s1), -0.5 * gs / torch.where(den == 0, 1.0, den)))
        c0 = actual < eta0 * pred
        c1 = actual < eta1 * pred
        c2 = actual < eta2 * pred
        nd = torch.where(c0, torch.minimum(torch.maximum(alpha, torch.full_like(alpha, s1)) * snorm, s2 * delta),
                         torch.where(c1, torch.maximum(s1 * delta, torch.minimum(alpha * snorm, s2 * delta)),
                                     torch.where(c2, torch.maximum(s1 * delta, torch.minimum(alpha * snorm,
                                                                                             s3 * delta)),
                                                 torch.maximum(delta, torch.minimum(alpha * snorm, s3 * delta)))))
        delta = torch.where(active, nd, delta)
        accept = active & (actual > eta0 * pred)
        f_prev = f
        W = torch.where(E(accept), W_new, W)
        f = torch.where(accept, f_new, f)
        g = torch.where(E(accept), g_new, g)
        it = it + accept.long()
        fails = torch.where(accept, torch.zeros_like(fails), fails + active.long())
        not_improving = active & ~accept & (fails >= max_fail)
        rc = conv.check(it, f, f_prev, g, accept, not_improving)
        newly_done = active & (rc > 0)
        reason = torch.where(newly_done, rc, reason)
        active &= ~newly_done
        fails = torch.where(accept, torch.zeros_like(fails), fails)
    return BatchedResult(W, f, it, reason)


def batched_lbfgs(data, loss, l2: float, W0: torch.Tensor, tol: float = 1e-7,
                  max_iter: int = 100, m: int = 10, l1: float = 0.0, max_ls: int = 30,
                  frozen: Optional[torch.Tensor] = None) -> BatchedResult:
    """Vectorised L-BFGS (OWL-QN when ``l1 > 0``) with backtracking Armijo line search per entity."""
    W = W0.clone()
    B = data.n_batch
    E = data.bexp
    dev, dt = W.device, W.dtype
    owl = l1 > 0

    def adjust(Wc, fc, gc):
        if not owl:
            return fc, gc
        f_adj = fc + l1 * data.babs_sum(Wc)
        dplus, dminus = gc + l1, gc - l1
        pg0 = torch.where(dminus > 0, dminus, torch.where(dplus < 0, dplus, torch.zeros_like(gc)))
        pg = torch.where(Wc == 0, pg0, gc + l1 * torch.sign(Wc))
        return f_adj, pg

    f_s, g_s = data.value_grad(loss, W, l2)
    if bool((W0 == 0).all()):
        f0z, g0z = f_s, g_s
    else:
        f0z, g0z = data.value_grad(loss, torch.zeros_like(W), l2)
    conv = _Convergence(data, f0z, g0z, tol, max_iter, dev)
    f, g = adjust(W, f_s, g_s)
    S = [torch.zeros_like(W) for _ in range(m)]  # history slot k: k-th most recent pair (slot 0 newest)
    Y = [torch.zeros_like(W) for _ in range(m)]
    rho = torch.zeros(B, m, dtype=dt, device=dev)
    hist = torch.zeros(B, dtype=torch.long, device=dev)  # number of valid pairs
    it = torch.zeros(B, dtype=torch.long, device=dev)
    reason = torch.zeros(B, dtype=torch.long, device=dev)
    active = _bn(data, g) > 0
    reason = torch.where(~active, torch.full_like(reason, 4), reason)
    if frozen is not None:
        active &= ~frozen
        reason = torch.where(frozen, torch.zeros_like(reason), reason)
    for _ in range(max_iter + 2):
        if not bool(active.any()):
            break
        # two-loop recursion; slot k holds the k-th most recent pair (slot 0 newest)
        q = g.clone()
        alphas = []
        for k in range(m):
            valid = (hist > k).to(dt)
            a = valid * rho[:, k] * data.bdot(S[k], q)
            q = q - E(a) * Y[k]
            alphas.append(a)
        yy = data.bdot(Y[0], Y[0])
        scale = torch.where(hist > 0, 1.0 / (rho[:, 0] * yy).clamp(min=1e-300), torch.ones_like(yy))
        q = q * E(scale)
        for k in range(m - 1, -1, -1):
            valid = (hist > k).to(dt)
            b = valid * rho[:, k] * data.bdot(Y[k], q)
            q = q + E(alphas[k] - b) * S[k]
        dvec = -q
        if owl:
            dvec = torch.where(dvec * g < 0, dvec, torch.zeros_like(dvec))
        gd = data.bdot(g, dvec)
        bad = active & (gd >= 0)
        # reset history and use steepest descent where the direction is not a descent direction
        dvec = torch.where(E(bad), -g, dvec)
        hist = torch.where(bad, torch.zeros_like(hist), hist)
        gd = data.bdot(g, dvec)
        orthant = torch.where(W != 0, torch.sign(W), torch.sign(-g))
        t = torch.where(it == 0, 1.0 / _bn(data, dvec).clamp(min=1e-300), torch.ones_like(gd))
        shrink = torch.where(it == 0, torch.full_like(gd, 0.1 if owl else 0.5), torch.full_like(gd, 0.5))
        searching = active.clone()
        W_acc, f_acc, g_acc, fs_acc, gs_acc = W.clone(), f.clone(), g.clone(), f_s.clone(), g_s.clone()
        found = torch.zeros_like(active)
        for _ls in range(max_ls):
            if not bool(searching.any()):
                break
            Wt = W + E(t) * dvec
            if owl:
                Wt = torch.where(torch.sign(Wt) != orthant, torch.zeros_like(Wt), Wt)
            ft_s, gt_s = data.value_grad(loss, Wt, l2)
            ft, gt = adjust(Wt, ft_s, gt_s)
            ok = searching & torch.isfinite(ft) & (ft <= f + 1e-4 * t * gd)
            W_acc = torch.where(E(ok), Wt, W_acc)
            f_acc = torch.where(ok, ft, f_acc)
            g_acc = torch.where(E(ok), gt, g_acc)
            fs_acc = torch.where(ok, ft_s, fs_acc)
            gs_acc = torch.where(E(ok), gt_s, gs_acc)
            found |= ok
            searching &= ~ok
            t = torch.where(searching, t * shrink, t)
        moved = active & found
        s_new = W_acc - W
        y_new = gs_acc - g_s
        sy = data.bdot(s_new, y_new)
        upd = moved & (sy > 1e-300)
        # shift history (newest in slot 0)
        ue = E(upd)
        S = [torch.where(ue, s_new if k == 0 else S[k - 1], S[k]) for k in range(m)]
        Y = [torch.where(ue, y_new if k == 0 else Y[k - 1], Y[k]) for k in range(m)]
        rho = torch.where(upd[:, None], torch.cat([(1.0 / sy.clamp(min=1e-300)).unsqueeze(1), rho[:, :-1]], 1), rho)
        hist = torch.where(upd, (hist + 1).clamp(max=m), hist)
        f_prev = f
        W = torch.where(E(moved), W_acc, W)
        f = torch.where(moved, f_acc, f)
        g = torch.where(E(moved), g_acc, g)
        f_s = torch.where(moved, fs_acc, f_s)
        g_s = torch.where(E(moved), gs_acc, g_s)
        it = it + moved.long()
        not_improving = active & ~found
        rc = conv.check(it, f, f_prev, g, moved, not_improving)
        newly = active & (rc > 0)
        reason = torch.where(newly, rc, reason)
        active &= ~newly
    return BatchedResult(W, f, it, reason)
