"""Row-space (kernel) re-parametrisation of wide per-entity random-effect problems.

A random-effect entity typically has few rows and many projected features (BASELINE config 5: n_e = 20 rows,
d_e = 1001 coefficients). Every vector of the reference's per-entity TRON / L-BFGS then has d_e entries although
the iterates live in an n_e-dimensional subspace: starting from w0 in the row space of X_e, the gradient
X_e^T (w l') + l2 w, every Hessian-vector product X_e^T D X_e v + l2 v and therefore every CG direction, trial
point and L-BFGS update stay in row(X_e).

With the Gram matrix K_e = X_e X_e^T = L_e L_e^T (Cholesky), Q_e = L_e^{-1} X_e has orthonormal rows and spans
row(X_e), so w = Q_e^T beta is an ISOMETRY from R^{n_e} onto the row space:

    margins  X_e w = X_e X_e^T L^{-T} beta = L_e beta        ||w||^2 = ||beta||^2       (Q Q^T = I)

i.e. the entity's problem is EXACTLY a dense GLM with the n_e x n_e design matrix L_e and the same L2 weight;
the optimizer iterates map one-to-one (w_k = Q^T beta_k), so TRON / L-BFGS take the same steps and stop on the
same Photon convergence tests as the primal solve (same f, same ||g||), in exact arithmetic. Requirements
checked by :func:`row_space_eligible`: L2 or no regularization (L1 breaks the row-space argument), no box
constraints, K_e positive definite (entities with linearly dependent rows stay on the primal path), warm start
inside the row space (the previous coordinate-descent solution always is; an external model is projected, which
changes only the iterates, not the optimum).

Cost: K_e for all entities takes 2 x n_max passes of the block-diagonal GLM kernels (column j of every K_e is
X (X^T e_j): an indicator per-row vector through the transpose then the forward kernel — deterministic, fp64,
no new kernels), once per dataset; each solve then touches B x n^2 doubles (4 GB at config 5) instead of the
D_total = 1.25e9-coefficient vectors, and the model returns to the primal space with one transpose pass
(w = X^T L^{-T} beta).
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from .batched import BatchedGLMData, BatchedResult, batched_lbfgs, batched_tron


def _bmv(A: torch.Tensor, x: torch.Tensor, trans: bool = False) -> torch.Tensor:
    """Batched small dense mat-vec (A [B, n, n] or A^T) x [B, n] (HIP kernel on the device, torch on the host)."""
    from ..ops.native import batched_gemv
    return batched_gemv(A, x, trans)


def _tri_inverse_lower(L: torch.Tensor) -> torch.Tensor:
    """Inverse of a batch of lower-triangular matrices by forward substitution vectorised over the batch
    (n steps of elementwise ops). rocBLAS' batched trsv runs one tiny solve per launch slot — measured 123 ms
    for 250K 20x20 systems on MI355X, vs a few ms here — and the inverse is reused by every later projection."""
    B, n, _ = L.shape
    X = torch.zeros_like(L)
    eye = torch.eye(n, dtype=L.dtype, device=L.device)
    for i in range(n):
        acc = eye[i].expand(B, n)
        if i:
            acc = acc - (L[:, i, :i].unsqueeze(-1) * X[:, :i, :]).sum(1)
        X[:, i, :] = acc / L[:, i, i:i + 1]
    return X


def row_space_eligible(l1: float, constraints=None) -> bool:
    return l1 == 0 and not constraints


class RowSpaceBatch:
    """Entities of a :class:`SegmentedGLMData` with 0 < n_e <= min(nmax, d_e) and a positive-definite Gram
    matrix, as one dense padded batch ``L [B, n, n]`` (padding rows: weight 0, unit diagonal)."""

    def __init__(self, seg, nmax: int = 64):
        self.seg = seg
        dev = seg.y.device
        n_e = seg.row_ptr[1:] - seg.row_ptr[:-1]
        d_e = seg.col_ptr[1:] - seg.col_ptr[:-1]
        cand = (n_e > 0) & (n_e <= nmax) & (n_e <= d_e)
        ents = torch.nonzero(cand).squeeze(1)
        self.n_entities = seg.B
        if ents.numel() == 0:
            self.ents = ents
            self.B = 0
            return
        n = int(n_e[ents].max())
        ar = torch.arange(n, device=dev)
        ne = n_e[ents]
        valid = ar.unsqueeze(0) < ne.unsqueeze(1)                               # [B, n]
        rows = torch.where(valid, seg.row_ptr[ents].unsqueeze(1) + ar, torch.full_like(valid, -1, dtype=torch.long))
        N = seg.y.numel()
        K = torch.zeros(ents.numel(), n, n, dtype=torch.float64, device=dev)
        ind = torch.zeros(N, dtype=torch.float64, device=dev)
        for j in range(n):
            vj = valid[:, j]
            rj = rows[vj, j]
            ind.zero_()
            ind[rj] = 1.0
            u = seg.glm.rmatvec(ind)                  # every eligible entity's row j, at its own columns
            z = seg.glm.matvec(u)                      # (X_e X_e^T)[:, j] on the entity's rows
            K[:, :, j] = torch.where(valid, z[rows.clamp(min=0)], torch.zeros((), dtype=torch.float64, device=dev))
        del ind
        # non-eligible entities also received u components (rows of OTHER entities never mix: block diagonal)
        pad = (~valid).to(torch.float64)
        K = K + torch.diag_embed(pad)
        L, info = torch.linalg.cholesky_ex(K)
        ok = info == 0
        self.ents = ents[ok]
        self.B = int(self.ents.numel())
        self.n = n
        self.L = L[ok].contiguous()
        self.rows = rows[ok]
        self.valid = valid[ok]
        self.w = torch.where(self.valid, seg.w[self.rows.clamp(min=0)], torch.zeros((), dtype=torch.float64,
                                                                                   device=dev))
        self.y = torch.where(self.valid, seg.y[self.rows.clamp(min=0)], torch.zeros((), dtype=torch.float64,
                                                                                   device=dev))
        self.Linv = _tri_inverse_lower(self.L)                           # [B, n, n], lower
        self.mask = torch.zeros(seg.B, dtype=torch.bool, device=dev)   # entities handled here
        self.mask[self.ents] = True
        self.beta: Optional[torch.Tensor] = None                        # last solution (row-space coordinates)

    def _slots(self, per_row: torch.Tensor) -> torch.Tensor:
        return torch.where(self.valid, per_row[self.rows.clamp(min=0)],
                           torch.zeros((), dtype=per_row.dtype, device=per_row.device))

    def beta_from_primal(self, W: torch.Tensor) -> torch.Tensor:
        """Orthogonal projection of primal coefficients onto the row space: beta = L^{-1} X w."""
        z = self._slots(self.seg.glm.matvec(W))
        return _bmv(self.Linv, z)

    def to_primal(self, beta: torch.Tensor) -> torch.Tensor:
        """w = X^T L^{-T} beta for the handled entities (zeros elsewhere): one transpose pass."""
        alpha = _bmv(self.Linv, beta, trans=True)                        # L^{-T} beta
        r = torch.zeros(self.seg.y.numel(), dtype=torch.float64, device=beta.device)
        r[self.rows[self.valid]] = alpha[self.valid]
        return self.seg.glm.rmatvec(r)

    def margins(self, beta: torch.Tensor) -> torch.Tensor:
        """Per-row X w (no offsets) of the handled entities = L beta, in the segmented row order."""
        z = torch.zeros(self.seg.y.numel(), dtype=torch.float64, device=beta.device)
        z[self.rows[self.valid]] = _bmv(self.L, beta)[self.valid]
        return z

    def solve(self, loss, l2: float, optimizer: str, W0: Optional[torch.Tensor], tol: float, max_iter: int,
              reuse_beta: bool = True) -> BatchedResult:
        """Solve the handled entities; returns the batched result over the ``B`` row-space problems."""
        if reuse_beta and self.beta is not None:
            beta0 = self.beta
        elif W0 is not None and bool((W0 != 0).any()):
            beta0 = self.beta_from_primal(W0)
        else:
            beta0 = torch.zeros(self.B, self.n, dtype=torch.float64, device=self.L.device)
        o = self._slots(self.seg.o)
        if (optimizer == "TRON" and self.L.is_cuda and self.n <= 64 and getattr(loss, "loss_id", -1) in (0, 1, 2)
                and os.environ.get("PML_RS_FUSED_TRON", "1") != "0"):
            # whole per-entity TRON in one kernel, L resident in LDS (ops/csrc/glm_kernels.hip rs_tron_kernel)
            from ..ops.native import rs_tron
            beta, f, iters, reason = rs_tron(self.L, self.y, o, self.w, beta0, loss.loss_id, l2, tol, max_iter)
            res = BatchedResult(beta, f, iters, reason)
            self.beta = res.W
            return res
        data = BatchedGLMData(self.L, self.y, o, self.w)
        if optimizer == "TRON":
            res = batched_tron(data, loss, l2, beta0, tol, max_iter)
        else:
            res = batched_lbfgs(data, loss, l2, beta0, tol, max_iter)
        self.beta = res.W
        return res
