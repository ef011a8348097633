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
no new kernels), once per dataset; each solve then touches sum_e n_c(e)^2 doubles (4 GB at config 5, entities
grouped in size classes so a power-law size mix does not pad every problem to the largest) instead of the
D_total = 1.25e9-coefficient vectors, and the model returns to the primal space with one transpose pass
(w = X^T L^{-T} beta).
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from ..utils.timing import trace_range
from .batched import BatchedGLMData, BatchedResult, batched_lbfgs, batched_tron

# rs_tron problem order from the previous solve's iteration counts (PML_RS_ORDER=1). Off by default: measured
# slower at 1.25M x 20 (8.04-8.24 vs 7.73-8.00 ms in entity order; the scattered L loads cost more than the
# shorter wave tails gain, profiles/rs_tron_variants_v5_1p25M.log)
RS_ORDER = os.environ.get("PML_RS_ORDER", "0") == "1"


def _bmv(A: torch.Tensor, x: torch.Tensor, trans: bool = False) -> torch.Tensor:
    """Batched small dense mat-vec (A [B, n, n] or A^T) x [B, n] (HIP kernel on the device, torch on the host)."""
    from ..ops.native import batched_gemv
    return batched_gemv(A, x, trans)


def _btrsv(L: torch.Tensor, x: torch.Tensor, trans: bool = False, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Batched triangular solves L^-1 x / L^-T x with the classes' Cholesky factors (HIP kernel on the device). The
    factors are never inverted: an explicit inverse cost O(B n^3) at setup (75 ms for game5pl's n = 80 class) and a
    second n x n matrix per problem in HBM, for products needed only by the primal back-map and foreign warm starts."""
    from ..ops.native import batched_trsv
    return batched_trsv(L, x, trans, out=out)


def _canonical_csr(csr, dev):
    """The (indptr, columns, values) block-diagonal CSR on ``dev`` when every row's columns are strictly
    increasing (what the per-entity Gram kernel needs), else None."""
    if csr is None:
        return None
    nip, pos, val = (t.to(dev) for t in csr)
    if pos.numel() > 1:
        inc = pos[1:] > pos[:-1]
        starts = nip[1:-1]
        inc[starts[(starts > 0) & (starts < pos.numel())] - 1] = True   # a row's first entry may start lower
        if not bool(inc.all()):
            return None
    return nip.to(torch.int64), pos.to(torch.int64), val.to(torch.float64)


def row_space_eligible(l1: float, constraints=None) -> bool:
    return l1 == 0 and not constraints


# Size classes of the row-space batch: an entity with n_e rows joins the smallest class bound >= n_e and a class
# is padded to the largest n_e among its members (not to the bound). One padded batch over power-law entity
# sizes (most entities have a handful of rows, a few have 64) would cost every problem the largest n^2 in
# memory and in the fused kernel's lane group; per class the kernel uses G = pow2 >= n lanes per problem.
SIZE_CLASSES = (1, 2, 4, 8, 12, 16, 24, 32, 48, 64, 80, 96, 112, 128, 160, 192)
ROW_SPACE_NMAX = 192      # rs_tron_big_kernel / seg_gram_kernel limit (one wave per problem, packed L in LDS)
# class launch order: "desc" widest first; "asc"; "small_first" = classes of n <= RS_SMALL_N first, then widest
# first (the small classes then never run alone after a concurrent fused primal launch has finished)
RS_CLASS_ORDER = os.environ.get("PML_RS_CLASS_ORDER", "desc")
RS_CLASS_DESC = RS_CLASS_ORDER == "desc"
RS_SMALL_N = int(os.environ.get("PML_RS_SMALL_N", "12"))
# fused class launches spread over this many streams (the current one + RS_STREAMS - 1 more), classes assigned
# longest-first to the least-loaded stream by B n^2. Off by default: on game5pl one stream runs ~41 ms of class
# launches back to back next to the fused primal launch, yet two streams measured slower (RE 44.4-45.0 vs 43.6 ms,
# scripts/gpu_r5_s10.sh): the classes then also compete with each other for the CUs the primal launch leaves
RS_STREAMS = max(1, int(os.environ.get("PML_RS_STREAMS", "1")))
RS_BIG_NNZ_RATIO = float(os.environ.get("PML_RS_BIG_NNZ_RATIO", "0.6"))   # n > 64: mean row nnz >= ratio x n


class _SizeClass:
    """One padded dense batch of row-space problems: L [B, n, n] (padding rows: weight 0, unit diagonal)."""

    def __init__(self, ents, n, L, rows, valid, w, y, off):
        self.ents, self.n, self.L, self.rows, self.valid, self.w, self.y = ents, n, L, rows, valid, w, y
        self.B = int(ents.numel())
        self.off = off                                                   # offset in the packed beta vector

    def view(self, flat: torch.Tensor) -> torch.Tensor:
        return flat[self.off:self.off + self.B * self.n].view(self.B, self.n)

    def slots(self, per_row: torch.Tensor) -> torch.Tensor:
        return torch.where(self.valid, per_row[self.rows.clamp(min=0)],
                           torch.zeros((), dtype=per_row.dtype, device=per_row.device))


class RowSpaceBatch:
    """Entities of a :class:`SegmentedGLMData` with 0 < n_e <= min(nmax, d_e) and a positive-definite Gram
    matrix, as dense padded batches per size class (:data:`SIZE_CLASSES`). Row-space coefficients of all
    classes are packed into one flat vector (class after class, ``[B_c, n_c]`` row-major each); ``ents``,
    ``valid`` and the solver results follow the same order."""

    def __init__(self, seg, nmax: int = 64, csr=None):
        nmax = min(int(nmax), ROW_SPACE_NMAX)
        self.seg = seg
        dev = seg.y.device
        n_e = seg.row_ptr[1:] - seg.row_ptr[:-1]
        d_e = seg.col_ptr[1:] - seg.col_ptr[:-1]
        cand = (n_e > 0) & (n_e <= nmax) & (n_e <= d_e)
        if nmax > 64 and csr is not None:
            # beyond 64 rows a row-space CG step (two LDS-resident triangular mat-vecs, ~n^2 / 2 FMAs each) pays
            # only when the entity's rows are dense enough: measured break-even on game5pl-like entities at ~0.5 n
            # non-zeros per row (rs_tron_big_kernel 10.7 ms vs primal 9.8 ms for 65..128-row entities of 51
            # non-zeros, profiles/row_space_big_r4.md); sparser entities stay on the primal fused path
            nip = csr[0].to(n_e.device)
            ent_nnz = nip[seg.row_ptr[1:]] - nip[seg.row_ptr[:-1]]
            dense_enough = ent_nnz.double() >= RS_BIG_NNZ_RATIO * n_e.double() * n_e.double()
            cand &= (n_e <= 64) | dense_enough
        ents = torch.nonzero(cand).squeeze(1)
        self.n_entities = seg.B
        self.classes = []
        self.beta: Optional[torch.Tensor] = None                        # last solution (packed)
        self.mask = torch.zeros(seg.B, dtype=torch.bool, device=dev)   # entities handled here
        if ents.numel() == 0:
            self.ents = ents
            self.B = 0
            self.n = 0
            return
        ne_all = n_e[ents]
        bounds = torch.tensor([b for b in SIZE_CLASSES if b < nmax] + [nmax], device=dev)
        cls_of = torch.searchsorted(bounds, ne_all)                    # smallest bound >= n_e
        # class members in entity order: one stable sort by class, the class sizes in one readback, then the
        # per-class row / width / non-zero maxima in a second one (no boolean selection + sync per class)
        order = torch.argsort(cls_of, stable=True)
        ents_s, ne_s = ents[order], ne_all[order]
        from ..ops.native import sorted_counts
        cnt = sorted_counts(cls_of[order], bounds.numel()).tolist()
        de_s = d_e[ents_s]
        csr = _canonical_csr(csr, dev) if dev.type == "cuda" else None
        if csr is not None:
            enz_s = csr[0][seg.row_ptr[ents_s + 1]] - csr[0][seg.row_ptr[ents_s]]
        spans, lo = [], 0
        for c in cnt:
            spans.append((lo, lo + c))
            lo += c
        spans = [sp for sp in spans if sp[1] > sp[0]]
        stats = torch.stack([torch.stack([ne_s[a:b].max(), de_s[a:b].max()] +
                                         ([enz_s[a:b].max()] if csr is not None else []))
                             for a, b in spans]).tolist() if spans else []
        members = [(ents_s[a:b], ne_s[a:b], st) for (a, b), st in zip(spans, stats)]
        N = seg.y.numel()
        geo = []
        for e, ne, st in members:
            n = int(st[0])
            ar = torch.arange(n, device=dev)
            valid = ar.unsqueeze(0) < ne.unsqueeze(1)                  # [B_c, n]
            rows = torch.where(valid, seg.row_ptr[e].unsqueeze(1) + ar,
                               torch.full_like(valid, -1, dtype=torch.long))
            geo.append((e, n, valid, rows, None, ne, st))
        gram = trace_range("row-space: Gram matrices")
        gram.__enter__()
        # (class, members) whose Gram columns come from indicator passes: all of them without a canonical device
        # CSR, else only the entities too wide for seg_gram_kernel's LDS image (d_e > SEG_GRAM_DMAX)
        need_ind = []
        if csr is not None:
            # K_e straight from the block-diagonal CSR, one wave per entity (seg_gram_kernel)
            from ..ops.native import SEG_GRAM_DMAX, seg_gram
            for gi, (e, n, valid, rows, _, ne, st) in enumerate(geo):
                if int(st[1]) <= SEG_GRAM_DMAX:
                    geo[gi] = (e, n, valid, rows, seg_gram(e, n, seg.row_ptr, seg.col_ptr, *csr, dmax=int(st[1]),
                                                            maxnnz=int(st[2])), ne, st)
                    continue
                ok = d_e[e] <= SEG_GRAM_DMAX
                K = torch.zeros(e.numel(), n, n, dtype=torch.float64, device=dev)
                if bool(ok.any()):
                    K[ok] = seg_gram(e[ok], n, seg.row_ptr, seg.col_ptr, *csr)
                geo[gi] = (e, n, valid, rows, K, ne, st)
                need_ind.append((gi, torch.nonzero(~ok).squeeze(1)))
        else:
            geo = [(e, n, valid, rows, torch.zeros(e.numel(), n, n, dtype=torch.float64, device=dev), ne, st)
                   for e, n, valid, rows, _, ne, st in geo]
            need_ind = [(gi, None) for gi in range(len(geo))]
        n_max = max((geo[gi][1] for gi, _ in need_ind), default=0)
        ind = torch.zeros(N, dtype=torch.float64, device=dev) if n_max else None
        for j in range(n_max):
            # column j of every K_e at once: indicator on row j of every such entity with n_e > j
            ind.zero_()
            for gi, sel in need_ind:
                _, n, valid, rows, *_r = geo[gi]
                if j < n:
                    v, r = (valid, rows) if sel is None else (valid[sel], rows[sel])
                    ind[r[v[:, j], j]] = 1.0
            u = seg.glm.rmatvec(ind, build_multi=False)                # every entity's row j, at its own columns
            z = seg.glm.matvec(u)                      # (X_e X_e^T)[:, j] on the entity's rows
            for gi, sel in need_ind:
                _, n, valid, rows, K, *_r = geo[gi]
                if j < n:
                    v, r = (valid, rows) if sel is None else (valid[sel], rows[sel])
                    col = torch.where(v, z[r.clamp(min=0)], torch.zeros((), dtype=torch.float64, device=dev))
                    if sel is None:
                        K[:, :, j] = col
                    else:
                        K[sel, :, j] = col
            del u, z
        del ind
        gram.__exit__(None, None, None)
        # factors: one batched Cholesky launch per class (padding slots = identity); the pivots of every class are
        # checked with ONE readback, and only a class with a failed factor pays a boolean selection
        from ..ops.native import batched_cholesky
        infos = []
        for gi, (e, n, valid, rows, K, ne, st) in enumerate(geo):
            with trace_range(f"row-space: Cholesky n={n}"):
                _, info = batched_cholesky(K, ne)
            infos.append(info)
        all_ok = torch.stack([(i == 0).all() for i in infos]).tolist() if infos else []
        off = 0
        kept = []
        for (e, n, valid, rows, L, ne, st), info, good in zip(geo, infos, all_ok):
            if not good:
                ok = info == 0
                if not bool(ok.any()):
                    continue
                L, rows, valid, e = L[ok].contiguous(), rows[ok], valid[ok], e[ok]
            zero = torch.zeros((), dtype=torch.float64, device=dev)
            w = torch.where(valid, seg.w[rows.clamp(min=0)], zero)
            y = torch.where(valid, seg.y[rows.clamp(min=0)], zero)
            c = _SizeClass(e, n, L, rows, valid, w, y, off)
            off += c.B * n
            self.classes.append(c)
            kept.append(e)
        del geo
        self.ents = torch.cat(kept) if kept else ents[:0]
        self.B = int(self.ents.numel())
        self.n = max((c.n for c in self.classes), default=0)
        self.size = off
        self.mask[self.ents] = True
        self.valid = (torch.cat([c.valid.reshape(-1) for c in self.classes]) if self.classes
                      else torch.zeros(0, dtype=torch.bool, device=dev))
        self.rows = (torch.cat([c.rows.reshape(-1) for c in self.classes]) if self.classes
                     else torch.zeros(0, dtype=torch.long, device=dev))
        # packed slot -> row of the valid slots, once (margins / to_primal scatter with them: no boolean-mask
        # indexing, which costs a nonzero pass and a host synchronisation per call)
        self.vslot = torch.nonzero(self.valid).squeeze(1)
        self.vrow = self.rows[self.vslot]
        # the per-entity back-map (to_primal) reads only the handled entities' rows: a compact copy of them, not
        # the whole segmented CSR (which the dataset frees once the sub-problems are built)
        self._primal_csr = self._compact_csr(csr) if csr is not None else None
        # slot of every compact back-map row in the packed solution: the back-map gathers its row weights straight
        # from L^-T beta (no zero-filled per-row vector, scatter and gather over the whole coordinate)
        self._primal_slot = None
        if self._primal_csr is not None:
            slot_of_row = torch.full((seg.y.numel(),), -1, dtype=torch.int64, device=dev)
            slot_of_row[self.vrow] = self.vslot
            self._primal_slot = slot_of_row[self._primal_csr[-1]]
            del slot_of_row
        self._z = None            # (beta, packed margins L beta) written by the fused solve
        # the primal model (to_primal: one transpose pass over the block-diagonal data) is read once per model:
        # build its shard-wide one-launch transpose tables here, with the rest of the setup, instead of running
        # one launch per row chunk at every read (24 launches, 20.7 ms at config 5 vs one launch)
        # (not needed when the per-entity back-map covers every handled entity: rs_primal reads the compact copy)
        glm = getattr(seg, "glm", None)
        if (self._primal_csr is None and glm is not None and getattr(glm, "_multi_t", "unset") == "unset"
                and hasattr(glm, "_build_multi_t")):
            glm._build_multi_t()

    def _compact_csr(self, csr):
        """(ents, row_ptr, col_ptr, nip, pos, val, rows) for ``rs_primal`` over the handled entities' rows only,
        or None when an entity is too wide for its LDS accumulator. Entity k of the compact list is addressed as
        index 2k of interleaved range arrays: ``row_ptr[2k:2k+2]`` its compact rows, ``col_ptr[2k:2k+2]`` its
        coefficient range in the packed primal vector; ``rows`` maps compact rows back to segmented rows."""
        from ..ops.native import RS_PRIMAL_DMAX
        seg = self.seg
        if self.B == 0:
            return None
        ents = self.ents
        dev = ents.device
        c_lo, c_hi = seg.col_ptr[ents], seg.col_ptr[ents + 1]
        if bool(((c_hi - c_lo) > RS_PRIMAL_DMAX).any()):
            return None
        r_lo = seg.row_ptr[ents]
        ne = seg.row_ptr[ents + 1] - r_lo
        rcum = torch.zeros(self.B + 1, dtype=torch.int64, device=dev)
        torch.cumsum(ne, 0, out=rcum[1:])
        nr = int(rcum[-1])
        rows = torch.repeat_interleave(r_lo - rcum[:-1], ne, output_size=nr) + torch.arange(nr, device=dev)
        nip, pos, val = csr
        k0 = nip[rows]
        nk = nip[rows + 1] - k0
        nip_c = torch.zeros(nr + 1, dtype=torch.int64, device=dev)
        torch.cumsum(nk, 0, out=nip_c[1:])
        from ..ops.native import csr_gather_rows
        pos_c, val_c = csr_gather_rows(nip, pos, val, rows, nip_c)       # one gather kernel over the rows
        if int(seg.col_ptr[-1]) < 2 ** 31:
            pos_c = pos_c.to(torch.int32)          # 4 bytes less per entry of the (bandwidth-bound) back-map pass
        row_ptr = torch.stack([rcum[:-1], rcum[1:]], 1).reshape(-1)
        col_ptr = torch.stack([c_lo, c_hi], 1).reshape(-1)
        # trailing entries: the wrapper's range checks read the last element as the total
        row_ptr = torch.cat([row_ptr, rcum[-1:]])
        col_ptr = torch.cat([col_ptr, seg.col_ptr[-1:]])
        ents2 = torch.arange(self.B, dtype=torch.int64, device=dev) * 2
        return ents2, row_ptr, col_ptr, nip_c, pos_c, val_c, rows

    def _slots(self, per_row: torch.Tensor) -> torch.Tensor:
        """Packed per-slot values of a per-row vector (0 in padding slots, whose row index is -1)."""
        if (per_row.is_cuda and per_row.dtype == torch.float64 and per_row.is_contiguous()
                and self.rows.device == per_row.device):
            from ..ops.native import masked_gather
            return masked_gather(per_row, self.rows)            # one pass
        return torch.where(self.valid, per_row[self.rows.clamp(min=0)],
                           torch.zeros((), dtype=per_row.dtype, device=per_row.device))

    def beta_from_primal(self, W: torch.Tensor) -> torch.Tensor:
        """Orthogonal projection of primal coefficients onto the row space: beta = L^{-1} X w (packed)."""
        z = self._slots(self.seg.glm.matvec(W))
        return torch.cat([_btrsv(c.L, c.view(z)).reshape(-1) for c in self.classes])

    def _alpha(self, beta: torch.Tensor) -> Optional[torch.Tensor]:
        """L^-T beta for every class, written in place into one packed vector (no per-class results and
        concatenation). The classes' solves run back to back on one stream: spread over four streams they took
        the same 2.6 ms on game5pl (the batch is throughput-bound, not launch-bound; `profiles/materialize_r6.md`)."""
        if not self.classes:
            return None
        alpha = torch.empty_like(beta)
        for c in self.classes:
            _btrsv(c.L, c.view(beta), trans=True, out=c.view(alpha))
        return alpha

    def to_primal(self, beta: torch.Tensor, fill: bool = True) -> torch.Tensor:
        """w = X^T L^{-T} beta for the handled entities (zeros elsewhere): one transpose pass. ``fill=False``: the
        caller writes every coefficient outside the handled entities' ranges itself, so they are left unset (the
        zero fill of a model-sized vector: 0.8 ms on game5pl's 540M coefficients)."""
        alpha = self._alpha(beta)                                                               # L^-T beta
        pc = getattr(self, "_primal_csr", None)
        if pc is not None and alpha is not None:
            # per-entity back-map over the handled entities' rows only (rs_primal_kernel, one wave per entity, on
            # the compact copy of their rows); the shard-wide transpose pass read every entity's rows (9.0 ms on
            # game5pl)
            from ..ops.native import rs_primal
            ents2, row_ptr, col_ptr, nip, pos, val, rows = pc
            d_total = int(self.seg.col_ptr[-1])
            W = (torch.zeros if fill else torch.empty)(d_total, dtype=torch.float64, device=beta.device)
            rs_primal(ents2, row_ptr, col_ptr, nip, pos, val, alpha[self._primal_slot], W)
            return W
        r = torch.zeros(self.seg.y.numel(), dtype=torch.float64, device=beta.device)
        if alpha is not None:
            r[self.vrow] = alpha[self.vslot]
        return self.seg.glm.rmatvec(r, build_multi=False)     # once per update: no shard-wide tables

    def margins(self, beta: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Per-row X w (no offsets) of the handled entities = L beta, in the segmented row order (the fused solve's
        own margins when ``beta`` is its result: no pass over L). ``out``: a per-row vector to write the handled
        rows into (its other rows are left as they are); default a fresh zero vector."""
        z = torch.zeros(self.seg.y.numel(), dtype=torch.float64, device=beta.device) if out is None else out
        if self._z is not None and self._z[0] is beta:
            zs = self._z[1]
        else:
            zs = torch.cat([_bmv(c.L, c.view(beta)).reshape(-1) for c in self.classes]) if self.classes else beta
        z[self.vrow] = zs[self.vslot]
        return z

    def _warm_beta(self, W0: Optional[torch.Tensor], reuse_beta: bool) -> torch.Tensor:
        if reuse_beta and self.beta is not None:
            return self.beta
        if W0 is not None and bool((W0 != 0).any()):
            return self.beta_from_primal(W0)
        return torch.zeros(self.size, dtype=torch.float64, device=self.seg.y.device)

    def prepare(self, W0: Optional[torch.Tensor], reuse_beta: bool = True):
        """The solve's inputs, queued on the CURRENT stream: ``(beta, o)`` = a fresh copy of the warm start (the
        fused kernels solve in place in it) and the per-slot offsets. Lets a caller that runs :meth:`solve` on a
        side stream, concurrently with other work, do these passes first on an idle device (under a concurrent
        fused primal launch they ran on leftover CUs: ~14 ms instead of ~0.5 ms on game5pl)."""
        return self._warm_beta(W0, reuse_beta).clone(), self._slots(self.seg.o)

    def solve(self, loss, l2: float, optimizer: str, W0: Optional[torch.Tensor], tol: float, max_iter: int,
              reuse_beta: bool = True, prep=None) -> BatchedResult:
        """Solve the handled entities; returns the batched result over the ``B`` row-space problems (``W`` is
        the packed coefficient vector; ``iters`` / ``reason`` / ``f`` follow ``ents``). ``prep``: the result of
        :meth:`prepare` (then ``W0`` / ``reuse_beta`` are not used)."""
        dev = self.seg.y.device
        fused = (optimizer == "TRON" and self.seg.y.is_cuda and getattr(loss, "loss_id", -1) in (0, 1, 2)
                 and os.environ.get("PML_RS_FUSED_TRON", "1") != "0")
        if prep is not None:
            beta, o = prep              # solved in place: the warm start is already in ``beta``
            beta0 = beta
        else:
            beta0 = self._warm_beta(W0, reuse_beta)
            o = self._slots(self.seg.o)
            beta = torch.empty_like(beta0)
        zs = torch.empty_like(beta0) if fused else None
        fs, its, rcs = [], [], []
        res_of = {}
        # launch order: the widest classes first (fewest problems, longest per-problem chains: the launches that fill
        # the device worst go where a concurrent fused primal launch fills it, the many-problem classes last)
        if RS_CLASS_ORDER == "small_first":
            order_c = sorted(range(len(self.classes)),
                             key=lambda i: (self.classes[i].n > RS_SMALL_N, -self.classes[i].n))
        else:
            order_c = sorted(range(len(self.classes)), key=lambda i: -self.classes[i].n) if RS_CLASS_DESC else \
                range(len(self.classes))
        streams = [None]
        if fused and dev.type == "cuda" and RS_STREAMS > 1 and len(self.classes) > 1:
            main = torch.cuda.current_stream(dev)
            if getattr(self, "_streams", None) is None:
                self._streams = [torch.cuda.Stream(dev) for _ in range(RS_STREAMS - 1)]
            streams = [main] + self._streams
            for st in self._streams:
                st.wait_stream(main)                       # warm starts / offsets written on the caller's stream
                for t in (beta, beta0, o, zs):
                    if t is not None:          # zs: None off the fused path; beta0 may alias beta
                        t.record_stream(st)
            load = [0] * len(streams)
            lane = {}
            for ci in sorted(range(len(self.classes)), key=lambda i: -self.classes[i].B * self.classes[i].n ** 2):
                k = min(range(len(streams)), key=lambda j: load[j])
                lane[ci] = k
                load[k] += self.classes[ci].B * self.classes[ci].n ** 2

        def solve_class(ci):
            nonlocal zs
            c = self.classes[ci]
            b0, oc = c.view(beta0), c.view(o)
            if fused:
                # whole per-entity TRON in one kernel, L resident in LDS (ops/csrc/glm_kernels.hip rs_tron_kernel)
                from ..ops.native import rs_tron
                # waves group problems by the iteration counts of this class's previous solve (a wave waits for its
                # slowest problem); a scheduling hint only, the results do not depend on it
                order = getattr(c, "order", None) if RS_ORDER else None
                if order is not None and order.numel() != c.L.shape[0]:
                    order = None
                _, f, it, rc = rs_tron(c.L, c.y, oc, c.w, b0, loss.loss_id, l2, tol, max_iter, out=c.view(beta),
                                       order=order, zout=c.view(zs))
                if RS_ORDER:
                    c.order = torch.argsort(it, stable=True).to(torch.int32)
                return f, it, rc
            data = BatchedGLMData(c.L, c.y, oc, c.w)
            solver = batched_tron if optimizer == "TRON" else batched_lbfgs
            r = solver(data, loss, l2, b0, tol, max_iter)
            c.view(beta).copy_(r.W)
            zs = None
            return r.f, r.iters, r.reason

        for ci in order_c:
            st = streams[lane[ci]] if len(streams) > 1 else None
            if st is None or st is streams[0]:
                res_of[ci] = solve_class(ci)
            else:
                with torch.cuda.stream(st):
                    res_of[ci] = solve_class(ci)
                for t in res_of[ci]:
                    t.record_stream(streams[0])
        for st in streams[1:]:
            streams[0].wait_stream(st)
        for ci in range(len(self.classes)):
            f, it, rc = res_of[ci]
            fs.append(f)
            its.append(it)
            rcs.append(rc)
        res = BatchedResult(beta, torch.cat(fs) if fs and fs[0] is not None else None, torch.cat(its),
                            torch.cat(rcs))
        self.beta = res.W
        self._z = None if zs is None else (res.W, zs)
        return res
