"""Fused per-entity PRIMAL TRON for random-effect entities outside the row-space batch.

The reference runs one ``SingleNodeOptimizationProblem`` (TRON over the entity's local rows) per entity
(``photon-api/.../algorithm/RandomEffectCoordinate.scala:103-143``,
``photon-api/.../optimization/SingleNodeOptimizationProblem.scala:85-103``). Entities with few rows are solved
in their row space (``row_space.py``); the rest — 65 .. thousands of rows over up to ``FUSED_DMAX`` projected
coefficients — go here: ONE kernel launch per LDS size class (``re_tron_csr_kernel``,
``ops/csrc/re_kernels.hip``) runs every entity's complete TRON in its own workgroup, with the entity's
coefficient vectors in LDS and each Hessian-vector product a single read of its CSR rows. No host round trip,
no global pass per CG step, entities converge independently (a converged entity stops reading its rows), and
the margins of the solution come out of the solve. Tall-narrow entities (d_e <= 64) use ``re_tron_hess_kernel``
instead: the exact per-entity Hessian X_e^T D X_e formed once per outer iteration on the fp64 matrix cores
(``v_mfma_f64_16x16x4f64``) and kept in LDS, so truncated CG costs no pass over the rows at all.

Entities wider than ``FUSED_DMAX`` or longer than ``FUSED_MAX_ROWS`` stay on the block-diagonal pass path
(``batched.batched_tron`` over ``RandomEffectDataset.entity_subset``).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import torch

FUSED_DMAX = 2048                    # LDS per workgroup: (5 + 4) x dmax doubles (<= 147 KB of the CU's 160 KB)
FUSED_MAX_ROWS = int(os.environ.get("PML_RE_FUSED_MAX_ROWS", str(1 << 22)))
FUSED_LOSSES = (0, 1, 2)             # logistic, Poisson, squared (the twice-differentiable losses)
_CLASSES = (256, 512, 1024, 2048)    # LDS size classes (max coefficients per entity of a launch)
_HESS_CLASSES = (16, 32, 48, 64)     # tall-narrow entities: d_e padded to these, exact Hessian on the matrix cores
HESS_DMAX = 64 if os.environ.get("PML_RE_HESS", "1") != "0" else 0
# Register-resident kernel (re_tron_res_kernel): rows held in VGPRs, entities longer than one workgroup's rows split
# over a cluster of up to RES_KMAX workgroups. Measured on game5pl-like entities (profiles/re_resident_ab_r4.md):
# it halves the time of the LARGEST entities (64 largest alone: 29.5 -> 15.3 ms) but runs the small / mid ones at
# half the streaming kernel's throughput (8-wave barriers and per-wave accumulator combines dominate their short
# passes). Policy ``auto``: only entities whose single-workgroup streaming solve would outlast the whole streaming
# launch (more than 1/RES_TAIL_SHARE of the batch's non-zeros) go to clusters; ``force``: every eligible entity;
# ``0``: none.
RESIDENT = os.environ.get("PML_RE_RESIDENT", "auto")
RES_TAIL_SHARE = int(os.environ.get("PML_RE_RES_TAIL_SHARE", "256"))
RES_ROW_NNZ = 64
RES_KMAX = int(os.environ.get("PML_RE_RES_KMAX", "128"))


QUAD_MIN_ROW_NNZ = 12      # pad rows to whole quads when the mean row holds >= 12 entries (<= 25 % padding)
# warm starts bound ||g(0)|| by ||X_e||_F ||c|| instead of a row pass at zero (re_tron_lean_kernel; PML_RE_LAZY_G0=0:
# always the exact pass)
LAZY_G0 = os.environ.get("PML_RE_LAZY_G0", "1") != "0"


def pad_rows_to_quads(nip: torch.Tensor, lcol: torch.Tensor, val: torch.Tensor):
    """Rows padded to multiples of 4 entries with column 0 / value 0.0 (which add exactly nothing to a margin and
    exactly 0 to an accumulator): ``(nip, lcol, val)`` of the padded CSR. The lean kernel then reads every row as
    whole quads (row_pass_q); the other fused kernels read the padded rows unchanged."""
    dev = nip.device
    rn = nip[1:] - nip[:-1]
    pn = (rn + 3) // 4 * 4
    nip_p = torch.zeros_like(nip)
    torch.cumsum(pn, 0, out=nip_p[1:])
    nnz, nnz_p = int(nip[-1]), int(nip_p[-1])
    row = torch.repeat_interleave(torch.arange(rn.numel(), device=dev), rn, output_size=nnz)
    dst = nip_p[row] + (torch.arange(nnz, device=dev) - nip[row])
    lcol_p = torch.zeros(nnz_p, dtype=lcol.dtype, device=dev)
    val_p = torch.zeros(nnz_p, dtype=val.dtype, device=dev)
    lcol_p[dst] = lcol[:nnz]
    val_p[dst] = val[:nnz]
    return nip_p, lcol_p, val_p


def _launch_dmax(dm: int, de: torch.Tensor, is_h: bool) -> int:
    """LDS width of a launch: the class width, except that lean launches (dm <= 1024) take their widest entity
    rounded up to 8 — a 1008-wide lean workgroup needs 40.8 KB of LDS, so FOUR fit a CU (1024 wide: three)."""
    from ..ops.native import RE_LEAN_DMAX
    if is_h or dm > RE_LEAN_DMAX:
        return dm
    return min(dm, (int(de.max()) + 7) // 8 * 8)


def fused_enabled() -> bool:
    return os.environ.get("PML_RE_FUSED", "1") != "0"


def fused_eligible(loss, optimizer: str, l1: float, constraints, device) -> bool:
    """The fused primal TRON applies to TRON with L2 / no regularization on the GPU for the smooth losses."""
    return (fused_enabled() and optimizer == "TRON" and l1 == 0 and not constraints
            and torch.device(device).type == "cuda" and getattr(loss, "loss_id", -1) in FUSED_LOSSES)


@dataclass
class FusedResult:
    W: torch.Tensor          # packed coefficients of the batch's entities
    f: torch.Tensor          # [B] final objective
    iters: torch.Tensor      # [B]
    reason: torch.Tensor     # [B] reason codes (batched.REASON_CODES)
    z: torch.Tensor          # per batch row: x_i . w of the solution (no offset)
    err: Optional[torch.Tensor] = None   # device error flag of the register-resident launch (check_error)

    def check_error(self) -> None:
        """Raise if the register-resident launch reported a cluster wait timeout. Reads the device flag (a host
        synchronisation with the launch), so callers run it only after queueing their concurrent work."""
        if self.err is not None and int(self.err.item()) != 0:
            raise RuntimeError("register-resident random-effect TRON: a workgroup cluster wait timed out "
                               "(results invalid); rerun with PML_RE_RESIDENT=0")


class EntityTronBatch:
    """The entities of a segmented random-effect coordinate that the fused kernel solves.

    ``mask`` [E] bool: candidate entities (e.g. not handled in their row space). Entities with data and
    ``d_e <= FUSED_DMAX``, ``n_e <= FUSED_MAX_ROWS`` are taken (``self.mask``); ``ents`` / ``rows`` / ``cols``
    are their parent entity indices, parent row positions and parent coefficient positions."""

    def __init__(self, ds, mask: torch.Tensor):
        seg = ds.seg
        dev = seg.y.device
        n_e = seg.row_ptr[1:] - seg.row_ptr[:-1]
        d_e = seg.col_ptr[1:] - seg.col_ptr[:-1]
        # the kernels address an entity's entries with 32-bit offsets from its first entry
        csr = getattr(ds, "_seg_csr", None)
        e_nnz = None
        if csr is not None:
            nip_all = csr[0].to(dev)
            e_nnz = nip_all[seg.row_ptr[1:]] - nip_all[seg.row_ptr[:-1]]
        sel = mask.to(dev) & (n_e > 0) & (d_e > 0) & (d_e <= FUSED_DMAX) & (n_e <= FUSED_MAX_ROWS)
        if e_nnz is not None:
            sel &= e_nnz.to(dev) < (1 << 31)
        self.n_heavy = 0
        if RESIDENT == "auto" and dev.type == "cuda" and getattr(ds, "_seg_csr", None) is not None:
            # tail entities too long for one register-resident launch (more rows than RES_KMAX workgroups hold,
            # or wider than its LDS image): one streaming workgroup would outlast the whole launch, so they go to
            # the block-diagonal pass path (grid-wide passes, run on its own stream next to this launch)
            from ..ops.native import re_res_params
            cap, rdmax, grid = re_res_params()
            kmax = min(RES_KMAX, grid // 2)
            nip_all = ds._seg_csr[0].to(dev)
            en = nip_all[seg.row_ptr[1:]] - nip_all[seg.row_ptr[:-1]]
            stream = sel & (d_e > HESS_DMAX)
            if bool(stream.any()):
                tail = stream & (en * RES_TAIL_SHARE > int(en[stream].sum()))
                heavy = tail & (((n_e + cap - 1) // cap > kmax) | (d_e > rdmax))
                self.n_heavy = int(heavy.sum())
                sel &= ~heavy
        self.mask = sel
        self.ents = torch.nonzero(sel).squeeze(1)
        self.B = int(self.ents.numel())
        self.W: Optional[torch.Tensor] = None          # last solution (warm start of the next solve)
        if dev.type == "cuda":
            from ..ops.native import check_lds_add_order
            check_lds_add_order(dev)                   # row passes accumulate with same-address ds_add_f64
        if self.B == 0:
            return
        ne, de = n_e[self.ents], d_e[self.ents]
        self.row_ptr = torch.zeros(self.B + 1, dtype=torch.int64, device=dev)
        torch.cumsum(ne, 0, out=self.row_ptr[1:])
        self.col_ptr = torch.zeros(self.B + 1, dtype=torch.int64, device=dev)
        torch.cumsum(de, 0, out=self.col_ptr[1:])
        n_rows = int(self.row_ptr[-1])
        if dev.type == "cuda":
            # the batch's rows straight from the parent CSR by one gather kernel (entity-local int16 columns, rows
            # padded to whole quads when the lean kernel reads quads): no nnz-sized torch index / scatter chain
            from ..ops.native import csr_gather_rows
            row_sel, col_sel = ds.entity_rows(sel)
            pnip, ppos, pval = (t.to(dev) for t in ds._seg_csr)
            row_nnz = pnip[row_sel + 1] - pnip[row_sel]
            nnz = int(row_nnz.sum())
            self.quad = (nnz > 0 and nnz >= QUAD_MIN_ROW_NNZ * n_rows and os.environ.get("PML_RE_QUAD", "1") != "0"
                         and not bool((de <= HESS_DMAX).any()))
            plen = (row_nnz + 3) // 4 * 4 if self.quad else row_nnz
            nip = torch.zeros(n_rows + 1, dtype=torch.int64, device=dev)
            torch.cumsum(plen, 0, out=nip[1:])
            cbase = seg.col_ptr[seg.row_entity[row_sel]]               # parent column of the entity's local 0
            self.lcol, val = csr_gather_rows(pnip, ppos, pval, row_sel, nip, cbase, torch.int16)
            del cbase, plen
            if os.environ.get("PML_CHECK_KERNEL_INPUTS", "0") == "1" and nnz:
                assert int(self.lcol.min()) >= 0 and int(self.lcol.max()) < int(de.max()), "local column range"
            self.nip, self.val = nip, val
        else:
            nip, pos, val, row_sel, col_sel, _ = ds.entity_csr(sel)
            row_ent = torch.repeat_interleave(torch.arange(self.B, device=dev), ne, output_size=n_rows)
            row_nnz = nip[1:] - nip[:-1]
            nnz = int(nip[-1])
            nnz_ent = torch.repeat_interleave(row_ent, row_nnz, output_size=nnz)
            lcol = pos - self.col_ptr[nnz_ent]
            del nnz_ent, pos
            self.lcol = lcol.to(torch.int16)                 # read as uint16 by the kernel (d_e <= 2048)
            self.nip, self.val = nip, val
            # rows padded to whole quads for the lean kernel's 4-entry loads (when rows are long enough that the
            # padding costs little); the streaming and resident kernels read the padded rows unchanged
            # (not with tall-narrow launches: re_tron_tall_kernel stages rows by ASSIGNMENT into a dense block,
            # where a column-0 padding entry could overwrite the real column 0)
            self.quad = (nnz > 0 and nnz >= QUAD_MIN_ROW_NNZ * n_rows and os.environ.get("PML_RE_QUAD", "1") != "0"
                         and not bool((de <= HESS_DMAX).any()))
            if self.quad:
                self.nip, self.lcol, self.val = pad_rows_to_quads(self.nip, self.lcol, self.val)
                nip = self.nip
        self.rows, self.cols = row_sel, col_sel
        row_ent = torch.repeat_interleave(torch.arange(self.B, device=dev), ne, output_size=n_rows)
        self.y, self.w = seg.y[row_sel].contiguous(), seg.w[row_sel].contiguous()
        self.n_rows = n_rows
        self.nnz = nnz
        self.scr = torch.empty(4 * max(n_rows, 1), dtype=torch.float64, device=dev)
        self.gsc = torch.empty(int(self.col_ptr[-1]), dtype=torch.float64, device=dev)   # lean kernel: gradient
        # ||X_e||_F^2 per entity (the lean kernel's bound of the zero point's gradient norm on warm starts)
        self.xf2 = None
        if LAZY_G0 and dev.type == "cuda":
            ent_len = self.nip[self.row_ptr[1:]] - self.nip[self.row_ptr[:-1]]
            self.xf2 = torch.segment_reduce(self.val * self.val, "sum", lengths=ent_len).contiguous()
        # launch classes by LDS size; inside a class the largest entities first (they bound the launch's tail).
        # Entities of at most HESS_DMAX coefficients (tall: the row space took the wide ones) run the exact-Hessian
        # kernel (MFMA), the others the sparse Hessian-vector kernel.
        ent_nnz = (nip[self.row_ptr[1:]] - nip[self.row_ptr[:-1]])
        if nnz and int(ent_nnz.max()) >= (1 << 31):
            raise ValueError("an entity of the fused batch has >= 2^31 non-zeros (32-bit kernel offsets)")
        self.launches = []
        hess = de <= HESS_DMAX
        # register-resident tasks (one persistent launch): clusters (k > 1 workgroups) first, largest first
        self.res = None
        stream_sel = ~hess
        if RESIDENT != "0" and bool(stream_sel.any()):
            from ..ops.native import re_res_params
            cap, rdmax, grid = re_res_params()
            kmax = min(RES_KMAX, grid // 2)
            ent_maxrow = torch.zeros(self.B, dtype=torch.int64, device=dev).scatter_reduce_(
                0, row_ent, row_nnz, reduce="amax", include_self=True)
            k_e = (ne + cap - 1) // cap
            res = stream_sel & (de <= rdmax) & (ent_maxrow <= RES_ROW_NNZ) & (k_e <= kmax)
            if RESIDENT != "force":
                # tail entities only: one workgroup streaming such an entity would outlast the whole launch
                res &= ent_nnz * RES_TAIL_SHARE > int(ent_nnz[stream_sel].sum())
            if bool(res.any()):
                idx = torch.nonzero(res).squeeze(1)
                # clusters first (descending k), then single-workgroup entities by descending non-zeros
                key = k_e[idx] * (int(ent_nnz.max()) + 1) + ent_nnz[idx]
                idx = idx[torch.argsort(key, descending=True, stable=True)]
                kk = k_e[idx]
                t0 = torch.zeros(idx.numel() + 1, dtype=torch.int64, device=dev)
                torch.cumsum(kk, 0, out=t0[1:])
                n_cl_tickets = int(kk[kk > 1].sum())
                from ..ops.native import require_re_lib
                ws_n = int(require_re_lib().pml_re_res_ws_doubles(max(n_cl_tickets, 1)))
                self.res = dict(ent=idx.to(torch.int32).contiguous(), t0=t0.to(torch.int32).contiguous(),
                                ws=torch.empty(ws_n, dtype=torch.float64, device=dev), grid=grid,
                                n=int(idx.numel()), clusters=int((kk > 1).sum()), tickets=int(t0[-1]))
                stream_sel = stream_sel & ~res
        for classes, sel, is_h in ((_HESS_CLASSES, hess, True), (_CLASSES, stream_sel, False)):
            cls = torch.searchsorted(torch.tensor(classes, device=dev), de)
            for c, dm in enumerate(classes):
                idx = torch.nonzero(sel & (cls == c)).squeeze(1)
                if idx.numel() == 0:
                    continue
                order = idx[torch.argsort(ent_nnz[idx], descending=True, stable=True)]
                self.launches.append((_launch_dmax(dm, de[idx], is_h), order.to(torch.int32).contiguous(),
                                      bool(is_h)))

    def solve(self, loss, l2: float, W0: Optional[torch.Tensor], offsets: torch.Tensor, tol: float, max_iter: int,
              max_fail: int = 5, max_cg: int = 20) -> FusedResult:
        """Solve every entity of the batch from ``W0`` (packed over the batch's coefficients; None = the last
        solution, or zeros the first time). ``offsets``: per batch row."""
        from ..ops.native import re_tron_csr
        dev = self.y.device
        if W0 is None:
            W0 = self.W if self.W is not None else torch.zeros(int(self.col_ptr[-1]), dtype=torch.float64,
                                                                device=dev)
        W = W0.to(torch.float64).contiguous().clone()
        f = torch.empty(self.B, dtype=torch.float64, device=dev)
        iters = torch.empty(self.B, dtype=torch.int32, device=dev)
        reason = torch.empty(self.B, dtype=torch.int32, device=dev)
        z = torch.empty(self.n_rows, dtype=torch.float64, device=dev)
        off = offsets.to(dev, torch.float64).contiguous()
        assert off.numel() == self.n_rows
        err = None
        if self.res is not None:
            from ..ops.native import re_tron_res
            r = self.res
            err = re_tron_res(r["ent"], r["t0"], r["ws"], r["grid"], self.row_ptr, self.col_ptr, self.nip, self.lcol,
                              self.val, self.y, off, self.w, W, f, iters, reason, z, loss.loss_id, l2, tol, max_iter,
                              max_fail, max_cg)
        for dm, order, is_h in self.launches:
            re_tron_csr(order, self.row_ptr, self.col_ptr, self.nip, self.lcol, self.val, self.y, off, self.w,
                        self.scr, W, f, iters, reason, z, loss.loss_id, l2, tol, max_iter, max_fail, max_cg, dm,
                        hessian=is_h, gsc=self.gsc, quad=self.quad, xf2=self.xf2)
        self.W = W
        # the error flag stays on the device: reading it here would wait for the whole launch before the caller
        # can queue concurrent work (the row-space side stream); callers call FusedResult.check_error() later
        return FusedResult(W, f, iters.to(torch.long), reason.to(torch.long), z, err)


class DenseEntityTronBatch:
    """A dense size bucket ``X [B, n, d]`` (RANDOM / IDENTITY projections, or the dense layout of INDEX_MAP) solved
    by the same fused kernels: every entity's padded rows presented as dense CSR rows (column ids 0..d-1, padding
    rows carry weight 0), so d <= 64 buckets form the exact Hessian on the fp64 matrix cores and wider ones run
    the sparse Hessian-vector kernel — one launch per bucket instead of the batched-GEMM TRON's per-CG-step torch
    launches (``batched.batched_tron`` over ``BatchedGLMData``; same TRON semantics)."""

    def __init__(self, X: torch.Tensor, y: torch.Tensor, w: torch.Tensor):
        B, n, d = X.shape
        if d > FUSED_DMAX:
            raise ValueError(f"dense bucket of {d} coefficients exceeds FUSED_DMAX={FUSED_DMAX}")
        dev = X.device
        self.B, self.n, self.d = B, n, d
        ar = lambda k, step: torch.arange(k + 1, dtype=torch.int64, device=dev) * step
        self.row_ptr, self.col_ptr, self.nip = ar(B, n), ar(B, d), ar(B * n, d)
        self.lcol = torch.arange(d, dtype=torch.int16, device=dev).repeat(B * n)
        self.val = X.to(torch.float64).reshape(-1).contiguous()
        self.quad = d >= QUAD_MIN_ROW_NNZ and d > HESS_DMAX and os.environ.get("PML_RE_QUAD", "1") != "0"
        if self.quad:
            self.nip, self.lcol, self.val = pad_rows_to_quads(self.nip, self.lcol, self.val)
        self.y = y.to(torch.float64).reshape(-1).contiguous()
        self.w = w.to(torch.float64).reshape(-1).contiguous()
        self.scr = torch.empty(4 * max(B * n, 1), dtype=torch.float64, device=dev)
        hess = d <= HESS_DMAX
        classes = _HESS_CLASSES if hess else _CLASSES
        dm = next(c for c in classes if c >= d)
        self.launch = (_launch_dmax(dm, torch.tensor([d]), hess), torch.arange(B, dtype=torch.int32, device=dev),
                       hess)

    def solve(self, loss, l2: float, W0: torch.Tensor, offsets: torch.Tensor, tol: float, max_iter: int,
              max_fail: int = 5, max_cg: int = 20) -> FusedResult:
        """``W0`` [B, d]; ``offsets`` [B, n]. Returns W [B, d] and margins z [B, n] (no offset)."""
        from ..ops.native import re_tron_csr
        B, n, d = self.B, self.n, self.d
        dev = self.y.device
        W = W0.to(dev, torch.float64).reshape(-1).contiguous().clone()
        f = torch.empty(B, dtype=torch.float64, device=dev)
        iters = torch.empty(B, dtype=torch.int32, device=dev)
        reason = torch.empty(B, dtype=torch.int32, device=dev)
        z = torch.empty(B * n, dtype=torch.float64, device=dev)
        off = offsets.to(dev, torch.float64).reshape(-1).contiguous()
        dm, order, is_h = self.launch
        re_tron_csr(order, self.row_ptr, self.col_ptr, self.nip, self.lcol, self.val, self.y, off, self.w, self.scr,
                    W, f, iters, reason, z, loss.loss_id, l2, tol, max_iter, max_fail, max_cg, dm, hessian=is_h,
                    quad=self.quad)
        return FusedResult(W.view(B, d), f, iters.to(torch.long), reason.to(torch.long), z.view(B, n))
