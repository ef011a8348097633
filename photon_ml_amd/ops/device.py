"""HBM-resident GLM row shard evaluated by the HIP kernels (``ops/csrc/glm_kernels.hip``).

Layout of one feature shard on one GPU (SURVEY §7.1 "Data layout", MI355X-first):

* rows are split into CHUNKS of ``chunk_rows`` (default 2^20) rows;
* per chunk a CSR stream (segments = rows) for ``z = X w`` and a CSC stream (segments = columns, rows local to
  the chunk) for ``g = X^T r``. Processing the transpose chunk by chunk keeps the gathered per-row vector of the
  chunk (4 MB in fp32) resident in the XCD L2s / Infinity Cache instead of gathering across the whole shard;
* int32 indices everywhere (chunk-local), values in bf16 (``precision="bf16"``), fp32 or fp64;
* per chunk the static block decomposition (see the kernel header) built once on the host.

One function evaluation = for each chunk: fused forward (margin + loss + per-row coefficient + block stats),
then transpose accumulate into the fp64 gradient; the per-block stats are reduced deterministically at the end.
No atomics anywhere: results are bitwise reproducible run to run.
"""
from __future__ import annotations

import ctypes
import os
import threading
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import scipy.sparse as sp
import torch

from ..data.matrix import LabeledData
from .native import SegChunkDesc, check, require_glm_lib, stream_handle
from .reference import GLMComputable
from .tiled import DEFAULT_ITEM_ENTRIES, TLFwdChunk, TLTChunk, tl_supported
from ..utils.timing import phase, trace_range

# Set after a tiled build's host -> device upload: GameData.prefetch_shard's copy waits for it, so the two copies do
# not share the host link (concurrent, the fixed-effect upload took 164 -> 472 ms) and the prefetch overlaps the
# layout build's device work instead
H2D_GATE = threading.Event()

LAYOUTS = ("auto", "tiled", "segmented")


def resolve_layout(layout: str, dim: int, chunk_rows: int) -> str:
    """``auto`` -> tiled when the packing can represent the shape (PML_LAYOUT env overrides ``auto``)."""
    import os
    if layout == "auto":
        layout = os.environ.get("PML_LAYOUT", "auto")
    if layout not in LAYOUTS:
        raise ValueError(f"unknown layout {layout}")
    if layout == "auto":
        layout = "tiled" if tl_supported(dim, chunk_rows) else "segmented"
    if layout == "tiled" and not tl_supported(dim, chunk_rows):
        raise ValueError(f"tiled layout cannot pack dim={dim} with chunk_rows={chunk_rows}")
    return layout

PRECISIONS = {"bf16": 0, "f32": 1, "f64": 2}
VAL_DTYPE = {0: torch.bfloat16, 1: torch.float32, 2: torch.float64}
VEC_DTYPE = {0: torch.float32, 1: torch.float32, 2: torch.float64}

FWD_MARGIN, FWD_VALUE_GRAD, FWD_HV, FWD_DZZ, FWD_LS = 0, 1, 2, 3, 4


def _pad8(n: int) -> int:
    return ((n + 7) // 8) * 8 + 8


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


class SegChunk:
    """One segmented stream (CSR chunk or CSC chunk) resident on the device."""

    def __init__(self, seg_ptr: np.ndarray, idx: torch.Tensor, val: torch.Tensor, device, nb: Optional[int] = None,
                 maxseg: Optional[int] = None, forward: bool = False):
        """``forward=True`` for CSR (row) streams: their blocks hold at most ``pml_maxseg_fwd()`` rows."""
        lib = require_glm_lib()
        seg_ptr = np.ascontiguousarray(seg_ptr, dtype=np.int32)
        nseg = len(seg_ptr) - 1
        nb = nb or lib.pml_nb()
        maxseg = maxseg or (lib.pml_maxseg_fwd() if forward else lib.pml_maxseg())
        nblk, nlong, npart = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(lib.pml_build_blocks(seg_ptr.ctypes.data, nseg, nb, maxseg, None, ctypes.byref(nblk), None, None,
                                   ctypes.byref(nlong), ctypes.byref(npart)), "count blocks")
        blk = np.zeros(max(5 * nblk.value, 5), dtype=np.int32)
        long_seg = np.zeros(max(nlong.value, 1), dtype=np.int32)
        long_ptr = np.zeros(nlong.value + 1, dtype=np.int32)
        check(lib.pml_build_blocks(seg_ptr.ctypes.data, nseg, nb, maxseg, blk.ctypes.data, ctypes.byref(nblk),
                                   long_seg.ctypes.data, long_ptr.ctypes.data, ctypes.byref(nlong),
                                   ctypes.byref(npart)), "build blocks")
        self.nseg, self.nblk, self.nlong, self.npart = nseg, nblk.value, nlong.value, npart.value
        self.nnz = int(seg_ptr[-1])
        dev = torch.device(device)
        self.seg_ptr = torch.from_numpy(seg_ptr).to(dev)
        self.blk = torch.from_numpy(blk).to(dev)
        self.long_seg = torch.from_numpy(long_seg).to(dev)
        self.long_ptr = torch.from_numpy(long_ptr).to(dev)
        # kernels read 8-aligned windows: pad the streams
        n_pad = _pad8(self.nnz)
        if idx.numel() < n_pad:
            idx = torch.cat([idx.to(dev, torch.int32), torch.zeros(n_pad - idx.numel(), dtype=torch.int32, device=dev)])
        if val.numel() < n_pad:
            val = torch.cat([val.to(dev), torch.zeros(n_pad - val.numel(), dtype=val.dtype, device=dev)])
        self.idx = idx.contiguous()
        self.val = val.contiguous()
        self.desc = SegChunkDesc(self.blk.data_ptr(), self.nblk, self.seg_ptr.data_ptr(), self.nseg,
                                 self.idx.data_ptr(), self.val.data_ptr(), self.long_seg.data_ptr(),
                                 self.long_ptr.data_ptr(), self.nlong, self.npart)

    kind = "seg"

    @property
    def nstats(self) -> int:
        return self.nblk

    @property
    def parts_needed(self) -> int:
        return self.npart

    def nbytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in (self.seg_ptr, self.blk, self.long_seg, self.long_ptr,
                                                           self.idx, self.val))


# PML_TRON_STATS=1: (kept forward blocks, kept transpose items) fractions of every entity-masked table rebuild
MASK_STATS = [] if os.environ.get("PML_TRON_STATS") == "1" else None

# row-sampled copies (down-sampling): below this kept fraction the narrow rounds are filtered too (a narrow round
# costs ~80 of a wide round's ~352 texture-address cycles, so it pays to convert once fewer than ~23 % remain)
NARROW_FILTER_BELOW = float(os.environ.get("PML_DS_NARROW_FILTER_BELOW", "0.23"))

# keep the margin cache across offset changes (set_offsets shifts it); PML_OFFSET_SHIFT_CACHE=0 drops it instead
OFFSET_SHIFT_CACHE = os.environ.get("PML_OFFSET_SHIFT_CACHE", "1") != "0"


class VecKey:
    """Identity of the coefficient vector a cached device quantity (margins, w l'') was computed at. The same
    tensor object at the same version matches without touching the device (the optimizer hands the accepted point
    back unchanged); another tensor matches if its values equal the keyed tensor's (one device comparison and host
    sync), provided the keyed tensor has not been modified in place since (else: no match, the quantity is
    recomputed). Holds a reference, not a copy: an 8 MB device copy per accepted step at D = 1M was one of the
    L-BFGS iteration's copy launches."""

    __slots__ = ("src", "ver")

    def __init__(self, w: torch.Tensor):
        self.src = w
        self.ver = w._version

    @property
    def shape(self):
        return self.src.shape

    def matches(self, w: torch.Tensor) -> bool:
        if w is self.src and w._version == self.ver:
            return True
        if self.src._version != self.ver or self.src.shape != w.shape:
            return False
        return bool(torch.equal(self.src, w.to(self.src.device, self.src.dtype)))


def _window_align(chunk_rows: int, precision: str) -> int:
    """Column-window start alignment: the transpose tile width of the chunks (1 when not tiled)."""
    from .tiled import t_bits
    cb = t_bits(chunk_rows, precision == "f64")
    return 1 << cb if cb is not None else 1


class DeviceGLMData(GLMComputable):
    """GLM row shard on one GPU evaluated with the native kernels."""

    def __init__(self, csr: List[SegChunk], csc: List[SegChunk], row_starts: Sequence[int], y, offsets, weights,
                 dim: int, precision: str = "f64", device="cuda", old_of_new: Optional[torch.Tensor] = None):
        self.lib = require_glm_lib()
        self.device = torch.device(device)
        if self.device.type == "cuda":
            from .native import check_lds_add_order
            check_lds_add_order(self.device)       # the kernels' bitwise determinism premise (once per process)
        self.prec = PRECISIONS[precision]
        self.precision = precision
        self.vdt = VEC_DTYPE[self.prec]
        self.csr, self.csc = csr, csc
        self.row_starts = list(row_starts)  # len = n_chunks + 1
        self.n_rows = self.row_starts[-1]
        self.dim = int(dim)
        rdt = self.vdt
        self.y = torch.as_tensor(y, device=self.device).to(rdt).contiguous()
        self.o = torch.as_tensor(offsets, device=self.device).to(rdt).contiguous()
        self.wt = torch.as_tensor(weights, device=self.device).to(rdt).contiguous()
        n = self.n_rows
        self.coef = torch.zeros(max(n, 1), dtype=rdt, device=self.device)
        self.dzz = torch.zeros(max(n, 1), dtype=rdt, device=self.device)
        self.track_hessian = False
        self._dzz_key: Optional[torch.Tensor] = None
        self._dzz_shift = None
        # scratch
        self.layout = "tiled" if csr and csr[0].kind == "tl" else "segmented"
        self.col_lo = [0] * len(csr)  # per-chunk column window base (see from_labeled(col_windows=True))
        self.blk_off = np.cumsum([0] + [c.nstats for c in csr]).tolist()
        self.long_off = np.cumsum([0] + [getattr(c, "nlong", 0) for c in csr]).tolist()
        self.stats = torch.zeros(2 * max(self.blk_off[-1], 1), dtype=torch.float64, device=self.device)
        self.long_stats = torch.zeros(2 * max(self.long_off[-1], 1), dtype=torch.float64, device=self.device)
        maxpart = max([c.parts_needed for c in csr + csc] + [1])
        self.parts = torch.zeros(maxpart, dtype=torch.float64, device=self.device)
        self.red_scratch = torch.zeros(512, dtype=torch.float64, device=self.device)
        self.out2 = torch.zeros(2, dtype=torch.float64, device=self.device)
        self.n_passes = 0
        # Features are relabelled hottest-first on device (so the forward kernel's LDS hot table holds the most
        # frequent features); the permutation is applied to the D-vectors at the boundary, invisible to callers.
        self.old_of_new = None if old_of_new is None else old_of_new.to(self.device, torch.int64)
        if self.old_of_new is not None:
            self.new_of_old = torch.empty_like(self.old_of_new)
            self.new_of_old[self.old_of_new] = torch.arange(self.dim, device=self.device)
        if os.environ.get("PML_CHECK_KERNEL_INPUTS", "0") == "1":
            self.validate()

    def validate(self):
        """Host-side check of every invariant the HIP kernels index by (no GPU sanitizer on the target pool):
        block/item windows inside their streams, round-aligned interleaved windows, gather indices < the column
        window / chunk rows, LDS slots < 2^bits, row ranges inside the shard. Raises ValueError on violation.
        Enabled at construction with ``PML_CHECK_KERNEL_INPUTS=1`` (costs one host pass over the streams)."""
        from .tiled import il_phys
        for c, (f, t) in enumerate(zip(self.csr, self.csc)):
            if f.kind != "tl":
                continue
            m = self.row_starts[c + 1] - self.row_starts[c]
            b = f.blk.cpu().to(torch.int64)
            if f.nblk and (int(b[:, 0].min()) < 0 or int((b[:, 0] + b[:, 1]).max()) > m
                           or int(b[:, 1].max()) > (1 << f.rbits)):
                raise ValueError(f"chunk {c}: forward block rows out of range")
            q = 256 if f.il else 4   # the kernels read whole rounds (il) / whole quads
            end = b[:, 2] + (b[:, 3] - b[:, 2] + q - 1) // q * q if f.il else (b[:, 3] + 3) // 4 * 4
            if f.nblk and (int(b[:, 2].min()) < 0 or int(end.max()) > f.pack.numel()):
                raise ValueError(f"chunk {c}: forward block window outside the stream")
            if f.il and f.nblk and bool((b[:, 2] % 256 != 0).any()):
                raise ValueError(f"chunk {c}: interleaved forward windows not round-aligned")
            ncols = int(self.dim) - self.col_lo[c]
            self._validate_narrow(c, f, b, ncols, "forward")
            pk, _ = f.logical()                   # absolute (col << rbits) | row, also with wide-round bases
            p = pk.cpu().to(torch.int64)
            wb = getattr(f, "wbase", None)
            if wb is not None and wb.numel() and int(wb.min()) < 0:
                raise ValueError(f"chunk {c}: negative wide-round base")
            if p.numel() and int((p >> f.rbits).max()) >= ncols:
                raise ValueError(f"chunk {c}: forward gather index >= column window")
            counts = f.unit_counts().cpu()
            blk_rows = torch.repeat_interleave(b[:, 1], counts)
            if p.numel() and bool(((p & ((1 << f.rbits) - 1)) >= blk_rows).any()):
                raise ValueError(f"chunk {c}: forward LDS slot >= block rows")
            it = t.items.cpu().to(torch.int64)
            if t.nitems:
                if int(it[:, 1].min()) < 0 or int(it[:, 2].max()) > t.pack.numel():
                    raise ValueError(f"chunk {c}: transpose item window outside the stream")
                if int(it[:, 3].max()) >= max(t.nparts, 1) and t.nparts:
                    raise ValueError(f"chunk {c}: transpose partial-row slot out of range")
                self._validate_narrow(c, t, it, m, "transpose")
                tp, _ = t.logical()
                q = tp.cpu().to(torch.int64) & 0xFFFFFFFF
                if q.numel() and int((q >> t.cbits).max()) >= m:
                    raise ValueError(f"chunk {c}: transpose gather row >= chunk rows")
                cols = (torch.repeat_interleave(it[:, 0], t.unit_counts().cpu()) << t.cbits) + (q & ((1 << t.cbits) - 1))
                if q.numel() and int(cols.max()) >= t.dim:
                    raise ValueError(f"chunk {c}: transpose column >= dim")
        if self.parts.numel() < max([c.parts_needed for c in self.csr + self.csc] + [1]):
            raise ValueError("partial-row scratch too small")
        self._validate_multi()
        return True

    def _validate_multi(self):
        """The shard-wide launch tables (when built): every unit's stream window inside ITS chunk's streams,
        narrow ranges inside the chunk's narrow section, the partial-row scratch large enough."""
        mb = getattr(self, "_multi", None)
        if mb is not None and not isinstance(mb, str):
            t = self._multi_blk.cpu().to(torch.int64)
            for c, ch in enumerate(self.csr):
                r = t[t[:, 0] == c]
                if ch.il and r.shape[0] and (int(r[:, 3].min()) < 0 or int((r[:, 3] + (r[:, 4] - r[:, 3] + 255) // 256 * 256).max())
                                   > ch.pack.numel() or int(r[:, 7].max()) > ch.nbase.numel() * (ch.n_narrow_rounds > 0)):
                    raise ValueError(f"chunk {c}: shard-wide forward table outside the chunk's streams")
        mt = getattr(self, "_multi_t", None)
        if mt is not None and not isinstance(mt, str):
            if self.parts.numel() < mt.parts_needed:
                raise ValueError("partial-row scratch too small for the shard-wide transpose")
            t = mt.items.cpu().to(torch.int64)
            for c, ch in enumerate(self.csc):
                r = t[t[:, 0] == c]
                if ch.il and r.shape[0] and (int(r[:, 2].min()) < 0 or int((r[:, 2] + (r[:, 3] - r[:, 2] + 255) // 256 * 256).max())
                                   > ch.pack.numel() or int(r[:, 7].max()) > ch.nbase.numel() * (ch.n_narrow_rounds > 0)):
                    raise ValueError(f"chunk {c}: shard-wide transpose table outside the chunk's streams")

    @staticmethod
    def _validate_narrow(c: int, ch, table: torch.Tensor, xlen: int, what: str):
        """Narrow rounds: per-unit ranges consecutive inside the narrow stream, every key window
        [base, base + 64) inside the gathered vector."""
        if table.shape[0] == 0:
            return
        n_lo, n_hi = table[:, 4], table[:, 5]
        nrounds = ch.nbase.numel() if ch.n_narrow_rounds else 0
        if bool((n_hi < n_lo).any()) or int(n_hi.max()) > nrounds or bool((n_lo[1:] != n_hi[:-1]).any()):
            raise ValueError(f"chunk {c}: {what} narrow round ranges inconsistent")
        if nrounds:
            base = ch.nbase.cpu().to(torch.int64)
            if ch.npack.numel() < 256 * nrounds or ch.nval.numel() < 256 * nrounds:
                raise ValueError(f"chunk {c}: {what} narrow stream shorter than its rounds")
            if int(base.min()) < 0 or int(base.max()) + 64 > xlen:
                raise ValueError(f"chunk {c}: {what} narrow key window outside the gathered vector")

    # ------------------------------------------------------------------
    @staticmethod
    def from_labeled(data: LabeledData, device="cuda", precision: str = "f64", chunk_rows: int = 1 << 20,
                     relabel: bool = True, layout: str = "auto", item_entries: Optional[int] = None,
                     col_windows: bool = False):
        """``col_windows``: store each chunk in its own column window ``[min col, max col]`` (local column ids,
        pointer-offset vectors). Used by the block-diagonal random-effect problems, where a chunk of
        entity-sorted rows touches a narrow contiguous column range of a huge ``dim`` (implies no relabel)."""
        if col_windows:
            relabel = False
        prec = PRECISIONS[precision]
        vdt = VAL_DTYPE[prec]
        dev = torch.device(device)
        x = data.x.tocsr()
        n, d = x.shape
        if dev.type == "cuda" and n and resolve_layout(layout, d, chunk_rows) == "tiled":
            return DeviceGLMData._from_labeled_device(x, data, dev, precision, chunk_rows, relabel, item_entries,
                                                      col_windows)
        if hasattr(x, "to_scipy"):                      # DeviceCSR on the host-side (segmented) build path
            x = x.to_scipy()
        old_of_new = None
        from ..parallel.dist import is_dist
        shared = relabel and is_dist() and not col_windows
        if shared or (relabel and x.nnz > 0):
            counts = np.bincount(x.indices, minlength=d).astype(np.int64)
            if shared:
                # one feature order on every rank (summed counts): the data-parallel gradient all-reduce can then
                # be bucketed and overlapped with the transpose pass (DistributedGLMData.overlap)
                import torch.distributed as tdist
                from ..parallel.sharding import comm_device
                ct = torch.from_numpy(counts).to(comm_device())
                tdist.all_reduce(ct)
                counts = ct.cpu().numpy()
            old_of_new_np = np.argsort(-counts, kind="stable")
            new_of_old_np = np.empty(d, dtype=np.int64)
            new_of_old_np[old_of_new_np] = np.arange(d)
            x = sp.csr_matrix((x.data, new_of_old_np[x.indices], x.indptr), shape=x.shape)
            old_of_new = torch.from_numpy(old_of_new_np)
        starts = list(range(0, n, chunk_rows)) + [n]
        if n == 0:
            starts = [0, 0]
        csr, csc = [], []
        col_lo = []
        wins = []
        align = _window_align(chunk_rows, precision)
        for a, b in zip(starts[:-1], starts[1:]):
            xc = x[a:b]
            if col_windows and xc.nnz:
                lo, hi = int(xc.indices.min()), int(xc.indices.max()) + 1
                lo -= lo % align          # tile-aligned windows: the shard-wide transpose can use global tiles
            else:
                lo, hi = 0, d
            wins.append((lo, hi))
        dmax = max([hi - lo for lo, hi in wins] + [1])
        layout = resolve_layout(layout, dmax, chunk_rows)
        cbits = None
        if layout == "tiled" and not col_windows and item_entries is None:
            from .tiled import shard_t_config
            cbits, item_entries = shard_t_config(int(x.nnz), n, d, chunk_rows)
        for (a, b), (lo, hi) in zip(zip(starts[:-1], starts[1:]), wins):
            xc = x[a:b]
            col_lo.append(lo)
            if lo != 0 or hi != d:
                xc = sp.csr_matrix((xc.data, xc.indices - lo, xc.indptr), shape=(b - a, hi - lo))
            dc = hi - lo
            if layout == "tiled":
                rp = torch.from_numpy((xc.indptr - xc.indptr[0]).astype(np.int64)).to(dev)
                col = torch.from_numpy(xc.indices.astype(np.int64)).to(dev)
                val = torch.from_numpy(xc.data.astype(np.float64)).to(dev).to(vdt)
                csr.append(TLFwdChunk(rp, col, val, dc))
                csc.append(TLTChunk(rp, col, val, dc, chunk_rows, cbits=cbits, item_entries=item_entries))
                continue
            sp_ = (xc.indptr - xc.indptr[0]).astype(np.int32)
            csr.append(SegChunk(sp_, torch.from_numpy(xc.indices.astype(np.int32)),
                                torch.from_numpy(xc.data.astype(np.float64)).to(vdt), dev, forward=True))
            xt = xc.tocsc()
            xt.sort_indices()
            xc = xc.copy()
            csc.append(SegChunk(xt.indptr.astype(np.int32), torch.from_numpy(xt.indices.astype(np.int32)),
                                torch.from_numpy(xt.data.astype(np.float64)).to(vdt), dev))
        out = DeviceGLMData(csr, csc, starts, torch.from_numpy(data.y), torch.from_numpy(data.offsets),
                            torch.from_numpy(data.weights), d, precision, dev, old_of_new)
        out.col_lo = col_lo
        return out

    @staticmethod
    def _from_labeled_device(x, data: LabeledData, dev, precision: str, chunk_rows: int, relabel: bool,
                             item_entries: Optional[int], col_windows: bool):
        """Tiled shard from a host CSR: the arrays are uploaded once and the feature counts, the hottest-first
        relabel, the chunking, the column windows and the layout sorts all run on the device (the host path sliced
        the CSR per chunk with scipy: 6.7 of 14.6 s at GAME config 5)."""
        n, d = x.shape
        with phase("tiled build: upload"):
            if isinstance(x.indptr, torch.Tensor):        # a DeviceCSR (entity-placed / routed rows): no host copy
                indptr, col, val = x.indptr.to(dev), x.indices.to(dev).to(torch.int64), x.data.to(dev)
            else:
                indptr = torch.from_numpy(np.ascontiguousarray(x.indptr, dtype=np.int64)).to(dev)
                col = torch.from_numpy(np.ascontiguousarray(x.indices)).to(dev).to(torch.int64)
                val = torch.from_numpy(np.ascontiguousarray(x.data)).to(dev)
        H2D_GATE.set()          # the host link is free: a prefetched shard (GameData.prefetch_shard) may copy now
        old_of_new = None
        from ..parallel.dist import is_dist
        shared = relabel and is_dist() and not col_windows
        relabel_phase = phase("tiled build: hottest-first relabel")
        relabel_phase.__enter__()
        if shared or (relabel and col.numel() > 0):
            from .native import key_histogram
            counts = key_histogram(col, d)          # hot columns (intercept, Zipf head): LDS-aggregated counts
            if shared:
                import torch.distributed as tdist
                from ..parallel.sharding import comm_device
                ct = counts.to(comm_device())
                tdist.all_reduce(ct)
                counts = ct.to(dev)
            oon = torch.argsort(-counts, stable=True)
            non = torch.empty_like(oon)
            non[oon] = torch.arange(d, device=dev)
            col = non[col]
            old_of_new = (oon, non)
            del counts
        relabel_phase.__exit__(None, None, None)
        out = DeviceGLMData.from_device_csr(indptr, col, val, torch.from_numpy(data.y), torch.from_numpy(data.offsets),
                                            torch.from_numpy(data.weights), d, dev, precision, chunk_rows,
                                            item_entries=item_entries, col_windows=col_windows)
        if old_of_new is not None:
            out.old_of_new, out.new_of_old = old_of_new
        return out

    @staticmethod
    def from_device_csr(indptr: torch.Tensor, col: torch.Tensor, val: torch.Tensor, y, offsets, weights, dim: int,
                        device="cuda", precision: str = "f64", chunk_rows: int = 1 << 20,
                        item_entries: Optional[int] = None, col_windows: bool = False):
        """Tiled-layout shard built from device-resident CSR arrays: chunking, column windows, the forward
        block sort and the transpose tile sort all run on the device (no host round trip of the non-zeros)."""
        dev = torch.device(device)
        vdt = VAL_DTYPE[PRECISIONS[precision]]
        indptr = indptr.to(dev, torch.int64)
        col = col.to(dev, torch.int64)
        n = indptr.numel() - 1
        starts = list(range(0, n, chunk_rows)) + [n] if n else [0, 0]
        ip = indptr[torch.tensor(starts, device=dev)].tolist()
        wins = []
        align = _window_align(chunk_rows, precision)
        for i in range(len(starts) - 1):
            ea, eb = ip[i], ip[i + 1]
            if col_windows and eb > ea:
                lo, hi = torch.aminmax(col[ea:eb])
                lo = int(lo)
                wins.append((lo - lo % align, int(hi) + 1))   # tile-aligned (see _window_align)
            else:
                wins.append((0, dim))
        dmax = max([hi - lo for lo, hi in wins] + [1])
        if resolve_layout("auto", dmax, chunk_rows) != "tiled":
            raise ValueError(f"from_device_csr needs the tiled layout (window {dmax} columns)")
        cbits = None
        if not col_windows and item_entries is None:
            from .tiled import shard_t_config
            cbits, item_entries = shard_t_config(int(ip[-1] - ip[0]), n, dim, chunk_rows)
        csr, csc, col_lo = [], [], []
        chunk_phase = phase(f"tiled build: {len(wins)} chunk layouts")
        chunk_phase.__enter__()
        for i, (lo, hi) in enumerate(wins):
            a, b = starts[i], starts[i + 1]
            ea, eb = ip[i], ip[i + 1]
            rp = indptr[a:b + 1] - ea
            c = col[ea:eb] - lo if lo else col[ea:eb]
            v = val[ea:eb].to(dev).to(vdt)
            csr.append(TLFwdChunk(rp, c, v, hi - lo))
            csc.append(TLTChunk(rp, c, v, hi - lo, chunk_rows, cbits=cbits, item_entries=item_entries))
            col_lo.append(lo)
            del c, v
        chunk_phase.__exit__(None, None, None)
        out = DeviceGLMData(csr, csc, starts, y, offsets, weights, dim, precision, dev, None)
        out.col_lo = col_lo
        return out

    def nbytes(self) -> int:
        return sum(c.nbytes() for c in self.csr + self.csc)

    def row_sampled(self, keep: torch.Tensor) -> Optional["DeviceGLMData"]:
        """K20 work saving: a shard over the SAME rows whose streams hold only the entries of the rows with
        ``keep`` (bool / uint8 [n_rows]); None when the layout cannot be compacted (segmented or plain-order
        streams). The reference trains each down-sampled fixed-effect update on a physically smaller RDD
        (``DistributedOptimizationProblem.scala:145-160``); here the dropped rows keep their positions (zero
        weight, margins = offsets) and their entries leave the streams, so every pass costs ~rate of a full one.

        Built per update by ``tl_compact_kernel`` (two passes over the wide streams, no sort, one host sync for all
        chunks): every unit keeps its table slot and its kept wide entries; the narrow sections (the cheap rounds)
        are shared unfiltered (``tiled.RowCompaction``). Row vectors (labels, offsets, weights) are SHARED with
        this shard; margin caches are the copy's own."""
        from .tiled import RowCompaction, stream_ptr_table
        from .native import TLFwdMultiDesc
        if self.layout != "tiled" or not self.csr or not all(getattr(ch, "il", 0) for ch in self.csr + self.csc):
            return None
        if any(getattr(ch, "wbase", None) is not None for ch in self.csr):
            return None      # compaction moves wide entries across rounds: their per-round key bases would not hold
        keep = keep.to(self.device, torch.uint8).contiguous()
        assert keep.numel() >= self.n_rows
        n = self.n_rows
        # this shard's launch tables first: building them may grow the partial-row scratch the copy shares
        if getattr(self, "_multi", "unset") == "unset":
            self._build_multi()
        if getattr(self, "_multi_t", "unset") == "unset":
            self._build_multi_t()
        # few rows kept: filter the narrow rounds too (all-wide copy); else share them (see RowCompaction)
        frac = float(keep[:n].sum()) / max(n, 1)
        filt = frac < NARROW_FILTER_BELOW
        jobs = []
        for c in range(len(self.csr)):
            kc = keep[self.row_starts[c]: self.row_starts[c + 1]]
            jobs.append(RowCompaction(self.csr[c], kc, True, filt))
            jobs.append(RowCompaction(self.csc[c], kc, False, filt))
        sizes = torch.stack([torch.stack([j.total, j.kept]) for j in jobs]).tolist()    # one host sync
        out = [j.finish(int(t), int(k)) for j, (t, k) in zip(jobs, sizes)]
        view = DeviceGLMData(out[0::2], out[1::2], self.row_starts, self.y, self.o, self.wt, self.dim,
                             self.precision, self.device, None)
        view.col_lo = list(self.col_lo)
        view.old_of_new = self.old_of_new
        if self.old_of_new is not None:
            view.new_of_old = self.new_of_old
        view.sampled_from = self
        view.kept_fraction = frac
        view._frob_sq = self.frob_sq()    # the copy holds a subset of the entries: still an upper bound
        if getattr(self, "z_cache", None) is not None and getattr(self, "_z_key", None) is not None:
            # the copy starts from this shard's cached margins (exact for the kept rows; the dropped rows' margins
            # only ever meet weight 0): the update's first evaluation needs no forward pass
            view.enable_margin_cache()
            view.z_cache.copy_(self.z_cache)
            view.zd.copy_(self.zd)
            view._z_key, view._z_chain, view._tpend = self._z_key, self._z_chain, self._tpend
        # shard-wide launch tables of the copy from this shard's (same units, new stream windows): no host-side
        # rebuild per update
        if self._multi is not None:
            nb = self._multi_blk.clone()
            cb = torch.cat([ch.blk for ch in view.csr])
            nb[:, 3:5] = cb[:, 2:4]
            nb[:, 6:8] = cb[:, 4:6]
            view._multi_blk = nb
            view._multi_ptrs = stream_ptr_table(view.csr, self.device)
            view._multi = TLFwdMultiDesc(nb.data_ptr(), nb.shape[0], self._multi.rbits, view._multi_ptrs.data_ptr(),
                                         self._multi.il)
        view._multi_t = None if self._multi_t is None else self._multi_t.restreamed(view.csc)
        gb = getattr(self, "_gbuckets", None)
        if gb is not None and gb[1] is not None:
            view._gbuckets = (gb[0], [(mt.restreamed(view.csc), c0, c1) for mt, c0, c1 in gb[1]])
        # same unit tables -> the same partial-row scratch (used in stream order); assigned last, after every
        # table this shard built above could have grown it
        view.parts = self.parts
        if os.environ.get("PML_CHECK_KERNEL_INPUTS", "0") == "1":
            view.validate()
        return view

    def set_offsets_sum(self, base: torch.Tensor, part: torch.Tensor) -> bool:
        """:meth:`set_offsets` of ``base + part`` (fp64 device vectors of the shard's rows) in one fused pass
        (``offset_update_kernel``: the sum, the cast to the row precision and the cached-margin shift); False when
        the inputs do not qualify (then nothing was changed)."""
        n = self.n_rows
        if not (n > 0 and base.is_cuda and part.is_cuda and base.dtype == part.dtype == torch.float64
                and base.numel() == part.numel() == n == self.o.numel() and base.is_contiguous()
                and part.is_contiguous() and base.device == self.o.device == part.device):
            return False
        from .native import offset_update
        zc = getattr(self, "z_cache", None)
        shift = (zc is not None and getattr(self, "_z_key", None) is not None and self._z_chain + 1 < self.LS_REFRESH
                 and getattr(self, "_masked", None) is None and OFFSET_SHIFT_CACHE)
        offset_update(base, part, self.o, zc[:n] if shift else None)
        if shift:
            self._z_chain += 1
            self._ls_t0 = None
        else:
            self._z_key = None
        self._step_base = None
        self._dzz_key = None
        return True

    def set_offsets(self, offsets):
        new = torch.as_tensor(offsets, device=self.device).to(self.vdt)
        zc = getattr(self, "z_cache", None)
        if (zc is not None and getattr(self, "_z_key", None) is not None and self._z_chain + 1 < self.LS_REFRESH
                and getattr(self, "_masked", None) is None and OFFSET_SHIFT_CACHE):
            # GAME: the residual offsets change between coordinate updates while the fixed-effect coefficients do
            # not; the cached margins (offsets included) shift by the offset change (one elementwise pass) and
            # the next update starts without a forward pass over the non-zeros (reference: every
            # FixedEffectCoordinate update re-evaluates X w from scratch)
            n = self.n_rows
            zc[:n].add_(new[:n].to(torch.float64) - self.o[:n].to(torch.float64))
            self._z_chain += 1
            self._ls_t0 = None
        else:
            self._z_key = None
        self.o.copy_(new)
        self._step_base = None
        self._dzz_key = None          # cached w l''(z) depends on the margins, hence on the offsets

    def mark_weights_changed(self):
        """The row weights were rewritten in place (down-sampling): drop every cache that folds them in (w l'',
        the first trial's (F, D)); the cached margins do not depend on the weights and stay valid."""
        self._dzz_key = None
        self._ls_t0 = None

    # ---- margin-space line search (GLMObjective.margin_line_search / LBFGS): z(t) = z0 + t zd ----------------
    # State: the margins of the last accepted point are z0 + tpend * zd (the accepted step is materialised
    # lazily in the next direction pass); _z_key identifies that point.
    LS_REFRESH = 50  # recompute z0 with a forward pass after this many chained updates (bounds rounding drift)

    def enable_margin_cache(self):
        """Keep the margins of the last full evaluation (8 B/row) so a line search needs one forward pass for
        the direction (which also evaluates the first trial step) and one elementwise pass per further trial."""
        if getattr(self, "z_cache", None) is None:
            n = max(self.n_rows, 1)
            self.z_cache = torch.zeros(n, dtype=torch.float64, device=self.device)
            self.zd = torch.zeros(n, dtype=torch.float64, device=self.device)
            self.ls_stats = torch.zeros(2 * 4096, dtype=torch.float64, device=self.device)
            self.ls_out = torch.zeros(2, dtype=torch.float64, device=self.device)
            self._z_key, self._z_chain, self._tpend, self._ls_t0 = None, 0, 0.0, None
        return True

    def _z_valid_for(self, w_eff, shift) -> bool:
        key = getattr(self, "_z_key", None)
        return (key is not None and key[1] == float(shift) and self._z_chain < self.LS_REFRESH
                and key[0].matches(w_eff))

    def ls_begin(self, w0_eff, shift0, d_eff, d_shift, t0: float = 1.0, loss=None, alt: bool = False,
                 stats_out: Optional[torch.Tensor] = None) -> bool:
        """Direction pass (FWD_LS): zd = X d_eff + d_shift, materialises the pending step into z0, and evaluates
        the first trial t0 (F, D and the speculative gradient input coef = w l'(z(t0))).

        ``alt``: a SPECULATIVE pass (L-BFGS plans the next iteration before the current step is validated,
        ``optimization/lbfgs.py``): the margins are read from the current buffer pair and written to the other
        one, which becomes current, so :meth:`ls_restore` of an earlier :meth:`ls_checkpoint` gets the untouched
        pair back. Refused (False, nothing queued) when the margins would first need a forward pass or the layout
        has no shard-wide launch. ``stats_out``: 2 fp64 device values that receive the first trial's (F, D)."""
        if loss is None:
            return False
        if getattr(self, "z_cache", None) is None:
            if alt:
                return False
            self.enable_margin_cache()   # from now on every value+gradient pass also stores its margins
        if not self._z_valid_for(w0_eff, shift0):
            if alt:
                return False
            self.fwd_all(self._vec(w0_eff), FWD_MARGIN, 0, shift0, None, None, z_out=self.z_cache, with_offset=1,
                         stats=False)
            self._z_key, self._z_chain, self._tpend = (VecKey(w0_eff), float(shift0)), 0, 0.0
        if alt:
            from .native import KERNEL_CONFIG
            if getattr(self, "_multi", "unset") == "unset":
                self._build_multi()
            if (self._multi is None or not KERNEL_CONFIG.get("tl_multi", 1)
                    or getattr(self, "_masked", None) is not None):
                return False
        with trace_range("K1' direction pass (margins of d + first trial)"):
            if alt:
                zin, din = self.z_cache, self.zd
                if getattr(self, "_zalt", None) is None:
                    self._zalt = (torch.empty_like(zin), torch.empty_like(din))
                zout, dout = self._zalt
                self.lib.pml_set_ls_in(zin.data_ptr(), din.data_ptr())
            else:
                zout, dout = self.z_cache, self.zd
            self.lib.pml_set_ls_args(zout.data_ptr(), float(t0), float(self._tpend))
            try:
                self.fwd_all(self._vec(d_eff), FWD_LS, loss.loss_id, d_shift, self.coef, None, z_out=dout)
            finally:
                self.lib.pml_set_ls_args(None, 0.0, 0.0)
                if alt:
                    self.lib.pml_set_ls_in(None, None)
            if alt:
                self.z_cache, self.zd, self._zalt = zout, dout, (zin, din)
            self._tpend = 0.0
            self._ls_t0 = float(t0)
            self._coef_stale = False
            # local (F, D) at t0, on the device: read by the first ls_eval (the caller synchronises once, after
            # everything this iteration needs has been queued), copied device-to-device by ls_finish_packed
            if stats_out is None:
                stats_out = torch.empty(2, dtype=torch.float64, device=self.device)
            self._ls_t0_dev = self._reduce_stats(stats_out)
            self._ls_t0_host = None
        return True

    _LS_STATE = ("z_cache", "zd", "_zalt", "_tpend", "_ls_t0", "_ls_t0_dev", "_ls_t0_host", "_z_key", "_z_chain",
                 "_track_u", "_dzz_key", "_dzz_shift", "_coef_stale", "_step_base")

    def ls_checkpoint(self) -> dict:
        """The margin-space line-search state (which buffer pair is current, the pending step, the cached first
        trial, the margin key): host references only, no device work. See :meth:`ls_begin` (``alt``)."""
        return {k: getattr(self, k, None) for k in self._LS_STATE}

    def ls_restore(self, ck: dict, t0_host=None):
        """Back to a :meth:`ls_checkpoint` (speculative passes queued since then are abandoned: they wrote only the
        other buffer pair and scratch). The row vector ``coef`` may since have been overwritten, so the first
        trial's gradient input is recomputed if that step is accepted after all; ``t0_host``: the first trial's
        (F, D) already read back, so the line search does not read them again."""
        for k, v in ck.items():
            setattr(self, k, v)
        self._coef_stale = True
        if t0_host is not None and self._ls_t0 is not None:
            self._ls_t0_host = tuple(float(v) for v in t0_host)

    @property
    def _ls_t0_vals(self):
        if self._ls_t0_host is None:
            self._ls_t0_host = tuple(self._ls_t0_dev.tolist())
        return self._ls_t0_host

    def _ls(self, loss, t, final, out):
        dzz = self.dzz if (final and self.track_hessian and loss.twice_differentiable) else None
        check(self.lib.pml_ls_eval(self.prec, self.n_rows, float(t), loss.loss_id, self.z_cache.data_ptr(),
                                   self.zd.data_ptr(), self.y.data_ptr(), self.wt.data_ptr(), int(final),
                                   self.coef.data_ptr() if final else None, None if dzz is None else dzz.data_ptr(),
                                   self.ls_stats.data_ptr(), out.data_ptr(), stream_handle(self.device)), "ls_eval")

    def ls_eval(self, loss, t: float):
        if self._ls_t0 is not None and float(t) == self._ls_t0:
            return self._ls_t0_vals       # evaluated by the direction pass
        with trace_range("line-search trial (margin space)"):
            self._ls(loss, t, 0, self.ls_out)
            f, d = self.ls_out.tolist()
        return f, d

    def ls_gate_supported(self) -> bool:
        """The gated first-trial finish (:meth:`ls_finish_gated`) needs the shard-wide transpose launch."""
        from .native import KERNEL_CONFIG
        if getattr(self, "_multi_t", "unset") == "unset":
            self._build_multi_t()
        return (self._multi_t is not None and KERNEL_CONFIG.get("tl_multi", 1) and getattr(self, "_masked", None) is None
                and getattr(self, "_ls_t0", None) == 1.0 and not getattr(self, "_coef_stale", False)
                and getattr(self, "_ls_t0_dev", None) is not None and self.z_cache.is_cuda)

    def ls_finish_gated(self, loss, pre: torch.Tensor, f0: float, l2: float, c1: float, c2: float,
                        x0: torch.Tensor, d: torch.Tensor):
        """Queue, behind the direction pass, the strong-Wolfe decision on its first trial t = 1
        (``ls_gate_kernel``) and the accepted-step epilogue of :meth:`ls_finish_fused` at t = 1 with its transpose
        workgroups gated on that decision: returns ``(scalars, x, F, g)`` with ``scalars`` the host list [pre, F, D,
        accept] (ONE readback, queued before the gated pass and waited for right after queueing it). The host keeps (x, F, g) only if it accepts t = 1 too; otherwise it restores
        an :meth:`ls_checkpoint` taken before this call (the gated pass did no work)."""
        out = torch.empty(8, dtype=torch.float64, device=self.device)
        gate = torch.empty(1, dtype=torch.int32, device=self.device)
        check(self.lib.pml_ls_gate(pre.data_ptr(), self._ls_t0_dev.data_ptr(), float(f0), float(l2), float(c1),
                                   float(c2), out.data_ptr(), gate.data_ptr(), stream_handle(self.device)), "ls_gate")
        # the readback is queued BEFORE the gated pass: a blocking copy after it would wait for the whole pass
        host = getattr(self, "_gate_host", None)
        if host is None:
            host = self._gate_host = torch.empty(8, dtype=torch.float64, pin_memory=True)
        host[:7].copy_(out[:7], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.lib.pml_set_gate(gate.data_ptr())
        try:
            x, F, g = self.ls_finish_fused(loss, 1.0, x0, d, l2)
        finally:
            self.lib.pml_set_gate(None)
        self._gate_keep = gate          # alive until the gated launch has run (stream order)
        ev.synchronize()
        return host[:7].tolist(), x, F, g

    LS_MULTI_MAX = 6

    def ls_eval_many(self, loss, ts):
        """:meth:`ls_eval` at several step lengths (<= LS_MULTI_MAX) in one pass over the rows and one readback:
        list of (F, D), each bitwise the single-step result (``ls_eval_multi_kernel``)."""
        ts = [float(t) for t in ts]
        if not (0 < len(ts) <= self.LS_MULTI_MAX) or not self.z_cache.is_cuda:
            return [self.ls_eval(loss, t) for t in ts]
        with trace_range("line-search trials (margin space, one pass)"):
            need = len(ts) * 2 * 4096
            if getattr(self, "_ls_multi_stats", None) is None or self._ls_multi_stats.numel() < need:
                self._ls_multi_stats = torch.empty(self.LS_MULTI_MAX * 2 * 4096, dtype=torch.float64,
                                                   device=self.device)
            out = torch.empty(2 * len(ts), dtype=torch.float64, device=self.device)
            arr = (ctypes.c_double * len(ts))(*ts)
            check(self.lib.pml_ls_eval_multi(self.prec, self.n_rows, len(ts), arr, loss.loss_id,
                                             self.z_cache.data_ptr(), self.zd.data_ptr(), self.y.data_ptr(),
                                             self.wt.data_ptr(), self._ls_multi_stats.data_ptr(), out.data_ptr(),
                                             stream_handle(self.device)), "ls_eval_multi")
            v = out.tolist()
        return [(v[2 * k], v[2 * k + 1]) for k in range(len(ts))]

    def ls_finish_packed(self, loss, t: float, w_eff, shift, need_s: bool = True, start_reduce=None,
                         nb: int = 0) -> torch.Tensor:
        """Accepted step: gradient input coef = w l'(z(t)) (already there when t is the first trial), then ONLY
        the transpose pass: packed local [G | F | S]. z0 <- z(t) is deferred to the next direction pass."""
        with trace_range("K1 gradient at the accepted step (transpose pass)"):
            out = torch.zeros(self.dim + 2, dtype=torch.float64, device=self.device)
            if self._ls_t0 is not None and float(t) == self._ls_t0 and not getattr(self, "_coef_stale", False) \
                    and not (self.track_hessian and loss.twice_differentiable):
                out[self.dim] = self._ls_t0_dev[0]
                if need_s:
                    # one fp64-accumulating reduction over the stored coefficients (no fp64 copy of the row vector)
                    torch.sum(self.coef[: self.n_rows], dim=0, dtype=torch.float64, out=out[self.dim + 1])
            else:
                self._ls(loss, t, 1, out[self.dim:])
            self._tpend = float(t)
            self._ls_t0 = None
            self._track_u = False
            self._z_key, self._z_chain = (VecKey(w_eff), float(shift)), self._z_chain + 1
            if self.track_hessian and loss.twice_differentiable:
                self._dzz_key, self._dzz_shift = VecKey(w_eff), float(shift)
            if start_reduce is not None:
                start_reduce(out[self.dim:])
                self._packed_bucketed(self.coef, out[: self.dim], start_reduce, nb)
            else:
                G = self._grad_target(out)
                self.t_all(self.coef, G)
                self._grad_finish(G, out)
            self.n_passes += 1
            return out

    def ls_finish_fused(self, loss, t: float, x0: torch.Tensor, d: torch.Tensor, l2: float):
        """The accepted step of a margin line search with an identity normalization, in one epilogue launch after
        the transpose pass: returns ``(x, F, g)`` with ``x = x0 + t d``, ``F`` the data loss at x (0-d device
        tensor, no host synchronisation) and ``g = X^T coef + l2 x`` in coefficient order (``ls_step_grad_kernel``
        gathers the device-order transpose result). Same values as :meth:`ls_finish_device` followed by the
        objective's torch epilogue (x0 + t * d, gradient + l2 * x), which it replaces (5 launches -> 1)."""
        from .native import ls_step_grad
        with trace_range("K1 gradient at the accepted step (transpose pass)"):
            first = (self._ls_t0 is not None and float(t) == self._ls_t0 and not getattr(self, "_coef_stale", False)
                     and not (self.track_hessian and loss.twice_differentiable))
            if first:
                F = self._ls_t0_dev[0]
            else:
                tail = torch.empty(2, dtype=torch.float64, device=self.device)
                self._ls(loss, t, 1, tail)
                F = tail[0]
            g = getattr(self, "_gscr", None)
            if g is None or g.numel() != self.dim:
                g = self._gscr = torch.empty(self.dim, dtype=torch.float64, device=self.device)
            G = g.zero_()
            self.t_all(self.coef, G)
            x, grad = ls_step_grad(x0, d, t, G, self.new_of_old if self.old_of_new is not None else None, l2)
            self._tpend = float(t)
            self._ls_t0 = None
            self._track_u = False
            self._z_key, self._z_chain = (VecKey(x), 0.0), self._z_chain + 1
            if self.track_hessian and loss.twice_differentiable:
                self._dzz_key, self._dzz_shift = VecKey(x), 0.0
            self.n_passes += 1
            return x, F, grad

    def ls_finish_device(self, loss, t: float, w_eff, shift, need_s: bool = True):
        """:meth:`ls_finish_sums` with F and S left as 0-d device tensors (no host synchronisation)."""
        out = self.ls_finish_packed(loss, t, w_eff, shift, need_s)
        return out[self.dim], out[self.dim + 1], out[: self.dim]

    def ls_finish_sums(self, loss, t: float, w_eff, shift, need_s: bool = True):
        out = self.ls_finish_packed(loss, t, w_eff, shift, need_s)
        f, s_ = out[self.dim:].tolist()
        return f, s_, out[: self.dim]

    # ---- TRON trial point in margin space: margins(w + s) = z0 + sum_i alpha_i u_i ------------------------------
    def step_begin(self, w_eff, shift) -> bool:
        """Start a TRON step at ``w``: z0 <- margins at w (normally already cached by the last evaluation; after a
        rejected trial the base margins are still in z0), zd <- 0, and from now on every Hessian-vector pass also
        stores its direction margins u = X d_eff - d_eff.s (8 B/row, ``FwdArgs.z_out`` in FWD_HV mode) so that
        :meth:`step_add` can accumulate the step's margins. The trial point is then evaluated by
        ``ls_finish_packed(t=1)``: one elementwise pass + the transpose pass, no forward pass."""
        if getattr(self, "z_cache", None) is None:
            self.enable_margin_cache()
        n = max(self.n_rows, 1)
        if not self._z_valid_for(w_eff, shift):
            base = getattr(self, "_step_base", None)
            if (base is not None and base[0] is not None and base[0][1] == float(shift)
                    and base[1] < self.LS_REFRESH and base[0][0].matches(w_eff)):
                self._z_key, self._z_chain = base     # rejected trial: z0 still holds the margins at w
            else:
                self.fwd_all(self._vec(w_eff), FWD_MARGIN, 0, shift, None, None, z_out=self.z_cache, with_offset=1,
                             stats=False)
                self._z_key, self._z_chain = (VecKey(w_eff), float(shift)), 0
            self._tpend = 0.0
        if self._tpend:
            self.z_cache.add_(self.zd, alpha=self._tpend)   # materialise the accepted step
            self._tpend = 0.0
        self.zd.zero_()
        self._ls_t0 = None
        if getattr(self, "u_dir", None) is None:
            self.u_dir = torch.zeros(n, dtype=torch.float64, device=self.device)
        self._track_u = True
        self._step_base = (self._z_key, self._z_chain)
        return True

    def step_add(self, alpha: float):
        """zd += alpha * (direction margins of the last Hessian-vector pass)."""
        self.zd.add_(self.u_dir, alpha=float(alpha))

    def _u_out(self):
        return self.u_dir if getattr(self, "_track_u", False) else None

    def set_weights(self, weights):
        self.wt.copy_(torch.as_tensor(weights, device=self.device).to(self.vdt))
        self.mark_weights_changed()

    # ------------------------------------------------------------------
    def _rows(self, t: torch.Tensor, c: int) -> int:
        return t.data_ptr() + self.row_starts[c] * t.element_size()

    def _fwd(self, c: int, x: torch.Tensor, mode: int, loss_id: int, shift: float, coef: Optional[torch.Tensor],
             dzz: Optional[torch.Tensor], z_out: Optional[torch.Tensor] = None, with_offset: int = 0,
             stats: bool = True):
        ch = self.csr[c]
        st = self.stats.data_ptr() + 2 * 8 * self.blk_off[c] if stats else None
        xp = x.data_ptr() + self.col_lo[c] * x.element_size()
        if ch.kind == "tl":
            masked = getattr(self, "_masked", None)
            desc = masked[0][c] if masked is not None and isinstance(masked[0], list) else ch.desc
            check(self.lib.pml_tl_fwd(
                self.prec, ctypes.byref(desc), xp, mode, loss_id, float(shift),
                self._rows(self.y, c), self._rows(self.o, c), self._rows(self.wt, c),
                None if coef is None else self._rows(coef, c), None if dzz is None else self._rows(dzz, c),
                None if z_out is None else self._rows(z_out, c), with_offset, st, stream_handle(self.device)),
                "tl_fwd")
            return
        lst = self.long_stats.data_ptr() + 2 * 8 * self.long_off[c] if stats else None
        check(self.lib.pml_seg_fwd(
            self.prec, ctypes.byref(ch.desc), xp, mode, loss_id, float(shift),
            self._rows(self.y, c), self._rows(self.o, c), self._rows(self.wt, c),
            None if coef is None else self._rows(coef, c), None if dzz is None else self._rows(dzz, c),
            None if z_out is None else self._rows(z_out, c), with_offset, st, lst, self.parts.data_ptr(),
            stream_handle(self.device)), "seg_fwd")

    def _t(self, c: int, x: torch.Tensor, G: torch.Tensor, square: int = 0):
        ch = self.csc[c]
        gp = G.data_ptr() + self.col_lo[c] * G.element_size()
        if ch.kind == "tl":
            masked = getattr(self, "_masked", None)
            desc = ch.desc if masked is None else masked[1][c]
            check(self.lib.pml_tl_t(self.prec, ctypes.byref(desc), self._rows(x, c), square, gp,
                                    self.parts.data_ptr(), stream_handle(self.device)), "tl_t")
            return
        check(self.lib.pml_seg_t(self.prec, ctypes.byref(ch.desc), self._rows(x, c), square, gp,
                                 self.parts.data_ptr(), stream_handle(self.device)), "seg_t")

    def _build_multi(self):
        """One-launch forward over all TL chunks (block table {chunk, row_lo, nrows, e_lo, e_hi, col_lo, n_lo,
        n_hi})."""
        self._multi = None
        if not self.csr or any(ch.kind != "tl" for ch in self.csr) or len({ch.rbits for ch in self.csr}) != 1:
            return
        tabs = []
        for c, ch in enumerate(self.csr):
            b = ch.blk.to(torch.int64)
            t = torch.empty((b.shape[0], 8), dtype=torch.int64, device=b.device)
            t[:, 0] = c
            t[:, 1] = b[:, 0] + self.row_starts[c]
            t[:, 2:5] = b[:, 1:4]
            t[:, 5] = self.col_lo[c]
            t[:, 6:8] = b[:, 4:6]
            tabs.append(t)
        self._multi_blk = torch.cat(tabs).to(torch.int32).contiguous()
        from .tiled import stream_ptr_table
        self._multi_ptrs = stream_ptr_table(self.csr, self.device)
        from .native import TLFwdMultiDesc
        if len({ch.il for ch in self.csr}) != 1:
            return
        self._multi = TLFwdMultiDesc(self._multi_blk.data_ptr(), self._multi_blk.shape[0], self.csr[0].rbits,
                                     self._multi_ptrs.data_ptr(), self.csr[0].il)

    def _build_multi_t(self):
        """One-launch transpose over all chunks. Column-window chunks (block-diagonal random-effect problems) take
        part when their windows start on tile boundaries: each chunk's items are shifted to global column tiles,
        and a tile shared by two chunks' windows is combined like any split tile."""
        self._multi_t = None
        if not self.csc or any(ch.kind != "tl" for ch in self.csc) or len({ch.cbits for ch in self.csc}) != 1:
            return
        C = 1 << self.csc[0].cbits
        if any(lo % C for lo in self.col_lo):
            return
        from .tiled import TLTMulti
        self._multi_t = TLTMulti(self.csc, self.row_starts, self.dim,
                                 tile_offsets=[lo // C for lo in self.col_lo] if any(self.col_lo) else None)
        need = self._multi_t.parts_needed
        if need > self.parts.numel():
            self.parts = torch.zeros(need, dtype=torch.float64, device=self.device)

    def fwd_all(self, x, mode, loss_id, shift, coef, dzz, z_out=None, with_offset=0, stats=True):
        """Forward pass over every chunk: one launch in the tiled layout (``KERNEL_CONFIG['tl_multi']``),
        else one launch per chunk."""
        from .native import KERNEL_CONFIG
        self.n_fwd = getattr(self, "n_fwd", 0) + 1
        if getattr(self, "_multi", "unset") == "unset":
            self._build_multi()
        if self._multi is not None and KERNEL_CONFIG.get("tl_multi", 1):
            p = lambda t: None if t is None else t.data_ptr()
            masked = getattr(self, "_masked", None)
            desc = self._multi if masked is None or isinstance(masked[0], list) else masked[0]
            check(self.lib.pml_tl_fwd_multi(
                self.prec, ctypes.byref(desc), x.data_ptr(), mode, loss_id, float(shift), self.y.data_ptr(),
                self.o.data_ptr(), self.wt.data_ptr(), p(coef), p(dzz), p(z_out), with_offset,
                self.stats.data_ptr() if stats else None, stream_handle(self.device)), "tl_fwd_multi")
            return
        for c in range(len(self.csr)):
            self._fwd(c, x, mode, loss_id, shift, coef, dzz, z_out, with_offset, stats)

    def t_all(self, x, G, square: int = 0, build_multi: bool = True):
        """Transpose pass over every chunk: one launch + one shard-wide combine in the tiled layout
        (``KERNEL_CONFIG['tl_multi']``), else per chunk. ``build_multi=False``: use the shard-wide tables only if
        they exist already (a one-off product should not pay their host-side build: ~0.2 s for the 1.2M column
        tiles of a config-5 random-effect shard)."""
        from .native import KERNEL_CONFIG
        self.n_t = getattr(self, "n_t", 0) + 1
        if getattr(self, "_multi_t", "unset") == "unset":
            if not build_multi:
                for c in range(len(self.csc)):
                    self._t(c, x, G, square)
                return
            self._build_multi_t()
        # masked passes (entity masks) keep the per-chunk launches: their live flags follow the per-chunk item order
        if (self._multi_t is not None and KERNEL_CONFIG.get("tl_multi", 1)
                and getattr(self, "_masked", None) is None):
            check(self.lib.pml_tl_t_multi(self.prec, ctypes.byref(self._multi_t.desc), x.data_ptr(), square,
                                          G.data_ptr(), self.parts.data_ptr(), stream_handle(self.device)),
                  "tl_t_multi")
            return
        for c in range(len(self.csc)):
            self._t(c, x, G, square)

    # ---- entity-masked passes (block-diagonal random-effect problems, optimization/batched.py): the forward
    # skips row blocks and the transpose skips column tiles whose rows / columns all belong to entities that are
    # no longer iterating. Rows and columns are grouped by entity, so a skipped block or tile touches no live
    # entity's margins or gradient; skipped margins come back as zero and skipped gradient columns as zero (or as
    # whatever the caller's output held: callers read active entities only). The kernels take per-unit live
    # flags (a workgroup of a dead unit exits at once): one device pass computes every flag, no host sync, no
    # table rebuild.
    def entity_mask_geometry(self, row_entity: torch.Tensor, col_entity: torch.Tensor):
        """(first, last) entity of every forward block and of every transpose item / split tile, concatenated
        over the chunks (with host-side offsets); False when the layout does not support masked passes."""
        cached = getattr(self, "_mgeo", None)
        if cached is not None:
            return cached
        self._mgeo = False
        if getattr(self, "_multi", "unset") == "unset":
            self._build_multi()
        if (self.old_of_new is not None or not self.csc or any(ch.kind != "tl" for ch in self.csc + self.csr)
                or not self.n_rows):
            return False
        nr, nc = row_entity.numel(), col_entity.numel()
        rspan = lambda lo, cnt: (row_entity[lo.clamp(0, nr - 1)], row_entity[(lo + cnt - 1).clamp(0, nr - 1)])
        if self._multi is not None:
            blk = self._multi_blk.to(torch.int64)
            f0, f1 = rspan(blk[:, 1], blk[:, 2])
            f_off = [0, int(blk.shape[0])]
        else:                         # per-chunk forward tables {row_lo (chunk-local), nrows, ...}
            parts = [rspan(ch.blk[: ch.nblk, 0].to(torch.int64) + self.row_starts[c], ch.blk[: ch.nblk, 1].to(torch.int64))
                     for c, ch in enumerate(self.csr)]
            f0 = torch.cat([p[0] for p in parts])
            f1 = torch.cat([p[1] for p in parts])
            f_off = np.cumsum([0] + [int(ch.nblk) for ch in self.csr]).tolist()
        firsts, lasts, i_off, m_off = [], [], [0], [0]
        for c, ch in enumerate(self.csc):
            C = 1 << ch.cbits
            hi = self.col_lo[c] + ch.dim - 1
            for t in (ch.items[: ch.nitems, 0].to(torch.int64), ch.mt_tiles[: ch.nmt].to(torch.int64)):
                firsts.append(col_entity[(self.col_lo[c] + t * C).clamp(0, nc - 1)])
                lasts.append(col_entity[torch.clamp(self.col_lo[c] + (t + 1) * C - 1, max=hi).clamp(0, nc - 1)])
            i_off.append(i_off[-1] + int(ch.nitems) + int(ch.nmt))
            m_off.append(i_off[-2] + int(ch.nitems))          # start of this chunk's split tiles
        t0, t1 = torch.cat(firsts), torch.cat(lasts)
        self._mgeo = (f0, f1, f_off, t0, t1, i_off, m_off)
        return self._mgeo

    def set_entity_mask(self, active: Optional[torch.Tensor], geometry=None):
        """Restrict matvec / rmatvec to the blocks and tiles of the ``active`` entities (bool [n_entities]);
        None restores full passes."""
        self._masked = None
        if active is None or not geometry:
            return
        f0, f1, f_off, t0, t1, i_off, m_off = geometry
        dup = lambda d: type(d).from_buffer_copy(d)
        cs = torch.zeros(active.numel() + 1, dtype=torch.int32, device=active.device)
        torch.cumsum(active.to(torch.int32), 0, out=cs[1:])
        live_f = ((cs[f1 + 1] - cs[f0]) > 0).to(torch.uint8)
        live_t = ((cs[t1 + 1] - cs[t0]) > 0).to(torch.uint8)
        keep = [live_f, live_t]
        if self._multi is not None:
            fdesc = dup(self._multi)
            fdesc.live = live_f.data_ptr()
        else:
            fdesc = []
            for c, ch in enumerate(self.csr):
                d = dup(ch.desc)
                d.live = live_f.data_ptr() + f_off[c]
                fdesc.append(d)
        tdescs = []
        for c, ch in enumerate(self.csc):
            d = dup(ch.desc)
            d.live = live_t.data_ptr() + i_off[c]
            d.live_mt = live_t.data_ptr() + m_off[c + 1]
            tdescs.append(d)
        self._masked = (fdesc, tdescs, keep)
        if MASK_STATS is not None:
            MASK_STATS.append((float(live_f.float().mean()), float(live_t.float().mean())))

    # ---- gradient buckets: the transpose split into column-tile ranges so each range's all-reduce can start as
    # soon as that range is final (overlap of the C1 collective with the rest of the transpose pass)
    def grad_buckets(self, nb: int):
        """``nb`` shard-wide transpose launches over contiguous column-tile ranges of ~equal entry counts:
        list of (TLTMulti, col_lo, col_hi) in PERMUTED column order; None if the layout does not allow it."""
        cache = getattr(self, "_gbuckets", None)
        if cache is not None and cache[0] == nb:
            return cache[1]
        if getattr(self, "_multi_t", "unset") == "unset":
            self._build_multi_t()
        if self._multi_t is None or nb < 2:
            self._gbuckets = (nb, None)
            return None
        from .tiled import TLTMulti
        C = 1 << self._multi_t.cbits
        ntiles = (self.dim + C - 1) // C
        work = np.zeros(ntiles, np.int64)
        for ch in self.csc:
            it = ch.items[: ch.nitems].cpu().numpy().astype(np.int64)
            np.add.at(work, it[:, 0], it[:, 2] - it[:, 1])
        cum = np.cumsum(work)
        cuts = [0] + [int(np.searchsorted(cum, cum[-1] * k / nb, side="right")) for k in range(1, nb)] + [ntiles]
        cuts = sorted(set(min(max(c, 0), ntiles) for c in cuts))
        out = []
        for t0, t1 in zip(cuts[:-1], cuts[1:]):
            if t1 > t0:
                mt = TLTMulti(self.csc, self.row_starts, self.dim, tile_range=(t0, t1))
                out.append((mt, t0 * C, min(t1 * C, self.dim)))
                if mt.parts_needed > self.parts.numel():
                    self.parts = torch.zeros(mt.parts_needed, dtype=torch.float64, device=self.device)
        self._gbuckets = (nb, out)
        return out

    def _packed_bucketed(self, x, G, start_reduce, nb: int, square: int = 0):
        self.n_t = getattr(self, "n_t", 0) + 1
        for mt, c0, c1 in self.grad_buckets(nb):
            check(self.lib.pml_tl_t_multi(self.prec, ctypes.byref(mt.desc), x.data_ptr(), square, G.data_ptr(),
                                          self.parts.data_ptr(), stream_handle(self.device)), "tl_t_multi")
            start_reduce(G[c0:c1])

    def value_grad_packed_overlap(self, loss, w_eff, margin_shift, start_reduce, nb: int = 4) -> torch.Tensor:
        """As :meth:`value_grad_packed` but the gradient is produced in ``nb`` column buckets and
        ``start_reduce(slice)`` is called on each final slice (and on [F, S]) while the rest of the pass is still
        running. The result stays in the PERMUTED (hot-first) feature order: the caller reduces across ranks —
        which must share the permutation — then applies :meth:`_unperm`. Bitwise equal to the one-launch pass."""
        with trace_range("K1 value+grad pass (bucketed)"):
            out = torch.zeros(self.dim + 2, dtype=torch.float64, device=self.device)
            if self._zero_point(loss, w_eff):
                self._zero_coef(loss, margin_shift, out[self.dim:])
                start_reduce(out[self.dim:])
                self._packed_bucketed(self.coef, out[: self.dim], start_reduce, nb)
                self.n_passes += 1
                return out
            if self._cached_point(w_eff, margin_shift):
                self._ls(loss, self._tpend, 1, out[self.dim:])
                self._ls_t0 = None
                if self.track_hessian and loss.twice_differentiable:
                    self._dzz_key, self._dzz_shift = VecKey(w_eff), float(margin_shift)
                start_reduce(out[self.dim:])
                self._packed_bucketed(self.coef, out[: self.dim], start_reduce, nb)
                self.n_passes += 1
                return out
            x = self._vec(w_eff)
            dzz = self.dzz if (self.track_hessian and loss.twice_differentiable) else None
            zc = getattr(self, "z_cache", None)
            self.fwd_all(x, FWD_VALUE_GRAD, loss.loss_id, margin_shift, self.coef, dzz, z_out=zc)
            if zc is not None:
                self._z_key, self._z_chain, self._tpend, self._ls_t0 = (VecKey(w_eff),
                                                                         float(margin_shift)), 0, 0.0, None
            out[self.dim:] = self._reduce_stats()
            start_reduce(out[self.dim:])
            self._packed_bucketed(self.coef, out[: self.dim], start_reduce, nb)
            if dzz is not None:
                self._dzz_key = VecKey(w_eff)
                self._dzz_shift = float(margin_shift)
            self.n_passes += 1
            return out

    def hv_packed_overlap(self, loss, w_eff, margin_shift, v_eff, v_shift, start_reduce, nb: int = 4):
        with trace_range("K2 Hessian-vector pass (bucketed)"):
            self._ensure_dzz(loss, w_eff, margin_shift)
            out = torch.zeros(self.dim + 2, dtype=torch.float64, device=self.device)
            x = self._vec(v_eff)
            self.fwd_all(x, FWD_HV, loss.loss_id, v_shift, self.coef, self.dzz, z_out=self._u_out())
            out[self.dim:] = self._reduce_stats()
            start_reduce(out[self.dim:])
            self._packed_bucketed(self.coef, out[: self.dim], start_reduce, nb)
            self.n_passes += 1
            return out

    def perm_fingerprint(self) -> float:
        """Order-sensitive fingerprint of the feature relabelling (0 for none): ranks must agree before they
        reduce gradients in the permuted order."""
        if self.old_of_new is None:
            return 0.0
        k = torch.arange(self.dim, device=self.device, dtype=torch.float64)
        return float((self.old_of_new.to(torch.float64) * torch.sin(k * 0.618 + 0.1)).sum()) + 1.0

    def _reduce_stats(self, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        out = self.out2 if out is None else out
        st = stream_handle(self.device)
        check(self.lib.pml_reduce_stats(self.stats.data_ptr(), self.blk_off[-1], out.data_ptr(), 0,
                                        self.red_scratch.data_ptr(), st), "reduce")
        if self.long_off[-1] > 0:
            check(self.lib.pml_reduce_stats(self.long_stats.data_ptr(), self.long_off[-1], out.data_ptr(), 1,
                                            None, st), "reduce")
        elif self.blk_off[-1] == 0:
            out.zero_()
        return out

    def _vec(self, w: torch.Tensor) -> torch.Tensor:
        w = w.to(self.device)
        perm = self.old_of_new
        if (w.is_cuda and w.dtype == torch.float64 and w.dim() == 1 and w.is_contiguous()
                and (perm is None or (perm.device == w.device and perm.dtype == torch.int64))):
            from .native import perm_cast
            return perm_cast(w, perm, self.vdt)      # gather + cast in one launch
        if perm is not None:
            w = w[perm]
        return w.to(self.vdt).contiguous()

    def _unperm(self, g: torch.Tensor) -> torch.Tensor:
        return g if self.old_of_new is None else g[self.new_of_old]

    def _grad_target(self, out: torch.Tensor) -> torch.Tensor:
        """Where a transpose pass accumulates the D-vector result: ``out[:dim]`` itself, or (relabelled columns)
        a zeroed device-order scratch that :meth:`_grad_finish` gathers into ``out`` in ONE kernel."""
        if self.old_of_new is None:
            return out[: self.dim]
        g = getattr(self, "_gscr", None)
        if g is None or g.numel() != self.dim:
            g = self._gscr = torch.empty(self.dim, dtype=torch.float64, device=self.device)
        return g.zero_()

    def _grad_finish(self, G: torch.Tensor, out: torch.Tensor):
        if self.old_of_new is not None:
            torch.index_select(G, 0, self.new_of_old, out=out[: self.dim])

    # ------------------------------------------------------------------
    def value_grad_packed(self, loss, w_eff, margin_shift) -> torch.Tensor:
        """Device tensor [D + 2] = (G, F, S) — packed so a DP wrapper can all-reduce it in one RCCL call."""
        with trace_range("K1 value+grad pass"):
            return self._value_grad_packed(loss, w_eff, margin_shift)

    def _cached_point(self, w_eff, shift) -> bool:
        """The margins at ``w_eff`` are cached (z0 + t_pending zd): value + gradient need no forward pass."""
        return (getattr(self, "z_cache", None) is not None and getattr(self, "_masked", None) is None
                and self._z_valid_for(w_eff, shift))

    def _zero_point(self, loss, w_eff) -> bool:
        """``w_eff`` is the optimizer's all-zero tolerance point (tagged by Optimizer.start): margins = offsets."""
        return bool(getattr(w_eff, "_pml_zero", False)) and not (self.track_hessian and loss.twice_differentiable)

    def _zero_coef(self, loss, margin_shift, stats_out: torch.Tensor):
        """coef = w l'(o + shift) and (F, S) at w = 0 by one elementwise pass (``ls_eval_kernel`` at t = 0): the
        forward pass over the non-zeros would only add zeros to the offsets. The reference evaluates this point to
        set its tolerances (Optimizer.scala, Appendix C.7)."""
        n = self.n_rows
        o = self.o[:n]
        # fp64 offsets and no shift: the kernel reads them in place (it never writes z0 / zd)
        z0 = o if (o.dtype == torch.float64 and float(margin_shift) == 0.0 and o.is_contiguous()) else \
            o.to(torch.float64) + float(margin_shift)
        check(self.lib.pml_ls_eval(self.prec, n, 0.0, loss.loss_id, z0.data_ptr(), z0.data_ptr(), self.y.data_ptr(),
                                   self.wt.data_ptr(), 1, self.coef.data_ptr(), None, self.ls_stats_buf().data_ptr(),
                                   stats_out.data_ptr(), stream_handle(self.device)), "ls_eval(zero)")

    def frob_sq(self) -> torch.Tensor:
        """||X||_F^2 of the shard (sum of the squared stored values, fp64; 0-d device tensor, computed once)."""
        c = getattr(self, "_frob_sq", None)
        if c is None:
            # forward copy: every non-zero once (padding entries are 0); one fp64 dot per stream, summed in order
            parts = []
            for ch in self.csr:
                for v in (ch.val, getattr(ch, "nval", None)):
                    if v is not None and v.numel():
                        v64 = v.reshape(-1).to(torch.float64)
                        parts.append(torch.dot(v64, v64))
                        del v64
            c = torch.stack(parts).sum() if parts else torch.zeros((), dtype=torch.float64, device=self.device)
            self._frob_sq = c
        return c

    def zero_point_sums(self, loss, margin_shift) -> list:
        """[F, S, ||c||^2, ||X||_F^2] at w = 0 (c = w l'(offsets + shift)): one elementwise pass, one sync; the
        zero point's gradient bound of GLMObjective.zero_state_bound."""
        out = torch.empty(4, dtype=torch.float64, device=self.device)
        self._zero_coef(loss, margin_shift, out[:2])
        out[2] = torch.linalg.vector_norm(self.coef[: self.n_rows], dtype=torch.float64) ** 2
        out[3] = self.frob_sq()
        return out.tolist()

    def ls_stats_buf(self) -> torch.Tensor:
        buf = getattr(self, "ls_stats", None)
        if buf is None:
            self.ls_stats = buf = torch.zeros(2 * 4096, dtype=torch.float64, device=self.device)
        return buf

    def _value_grad_packed(self, loss, w_eff, margin_shift) -> torch.Tensor:
        out = (torch.zeros if self.old_of_new is None else torch.empty)(self.dim + 2, dtype=torch.float64,
                                                                        device=self.device)
        G = self._grad_target(out)
        if self._zero_point(loss, w_eff):
            self._zero_coef(loss, margin_shift, out[self.dim:])
            self.t_all(self.coef, G)
            self._grad_finish(G, out)
            self.n_passes += 1
            return out
        if self._cached_point(w_eff, margin_shift):
            self._ls(loss, self._tpend, 1, out[self.dim:])    # coef (+ w l'') and (F, S) from cached margins
            self._ls_t0 = None
            if self.track_hessian and loss.twice_differentiable:
                self._dzz_key, self._dzz_shift = VecKey(w_eff), float(margin_shift)
            self.t_all(self.coef, G)
            self._grad_finish(G, out)
            self.n_passes += 1
            return out
        x = self._vec(w_eff)
        dzz = self.dzz if (self.track_hessian and loss.twice_differentiable) else None
        zc = getattr(self, "z_cache", None)
        self.fwd_all(x, FWD_VALUE_GRAD, loss.loss_id, margin_shift, self.coef, dzz, z_out=zc)
        if zc is not None:
            self._z_key, self._z_chain, self._tpend, self._ls_t0 = (VecKey(w_eff), float(margin_shift)), \
                0, 0.0, None
        self.t_all(self.coef, G)
        out[self.dim:] = self._reduce_stats()
        self._grad_finish(G, out)
        if dzz is not None:
            self._dzz_key = VecKey(w_eff)
            self._dzz_shift = float(margin_shift)
        self.n_passes += 1
        return out

    def value_grad_sums(self, loss, w_eff, margin_shift):
        out = self.value_grad_packed(loss, w_eff, margin_shift)
        fs = out[self.dim:].tolist()
        return fs[0], fs[1], out[: self.dim]

    def _ensure_dzz(self, loss, w_eff, shift):
        key = self._dzz_key
        if key is not None and self._dzz_shift == float(shift) and key.matches(w_eff):
            return
        x = self._vec(w_eff)
        self.fwd_all(x, FWD_DZZ, loss.loss_id, shift, self.dzz, None, stats=False)
        self._dzz_key = VecKey(w_eff)
        self._dzz_shift = float(shift)

    def hv_packed(self, loss, w_eff, margin_shift, v_eff, v_shift) -> torch.Tensor:
        with trace_range("K2 Hessian-vector pass"):
            return self._hv_packed(loss, w_eff, margin_shift, v_eff, v_shift)

    def _hv_packed(self, loss, w_eff, margin_shift, v_eff, v_shift) -> torch.Tensor:
        self._ensure_dzz(loss, w_eff, margin_shift)
        out = (torch.zeros if self.old_of_new is None else torch.empty)(self.dim + 2, dtype=torch.float64,
                                                                        device=self.device)
        H = self._grad_target(out)
        x = self._vec(v_eff)
        self.fwd_all(x, FWD_HV, loss.loss_id, v_shift, self.coef, self.dzz, z_out=self._u_out())
        self.t_all(self.coef, H)
        out[self.dim:] = self._reduce_stats()
        self._grad_finish(H, out)
        self.n_passes += 1
        return out

    def hv_sums(self, loss, w_eff, margin_shift, v_eff, v_shift):
        out = self.hv_packed(loss, w_eff, margin_shift, v_eff, v_shift)
        return out[: self.dim], float(out[self.dim + 1])

    def hdiag_sums(self, loss, w):
        x = self._vec(w)
        out = torch.zeros(self.dim, dtype=torch.float64, device=self.device)
        self.fwd_all(x, FWD_DZZ, loss.loss_id, 0.0, self.coef, None, stats=False)
        self.t_all(self.coef, out, square=1)
        self._dzz_key = None
        return self._unperm(out)

    def matvec(self, w) -> torch.Tensor:
        """z = X w (fp64, no offsets)."""
        return self.margins(w, 0.0, False)

    def rmatvec(self, r, square: bool = False, build_multi: bool = True) -> torch.Tensor:
        """g = X^T r (``square``: (X.X)^T r) for a per-row vector r (fp64 result, original column order).
        ``build_multi=False`` for one-off products (see :meth:`t_all`)."""
        rr = torch.as_tensor(r, device=self.device).to(self.vdt).contiguous()
        if rr.numel() < max(self.n_rows, 1):
            rr = torch.cat([rr, torch.zeros(max(self.n_rows, 1) - rr.numel(), dtype=self.vdt, device=self.device)])
        out = torch.zeros(self.dim, dtype=torch.float64, device=self.device)
        self.t_all(rr, out, square=int(square), build_multi=build_multi)
        return self._unperm(out)

    def margins(self, w, margin_shift: float = 0.0, with_offsets: bool = False):
        if (getattr(self, "_masked", None) is None and getattr(self, "z_cache", None) is not None
                and isinstance(w, torch.Tensor) and self._z_valid_for(w, margin_shift)):
            # the margins of the optimizer's last accepted point are cached (z0 + t_pending zd, offsets included):
            # scoring the returned model needs no forward pass
            n = self.n_rows
            if self.z_cache.is_cuda and self.o.dtype in (torch.float32, torch.float64):
                from .native import cached_margins           # one pass instead of clone / add_ / cast / sub_
                return cached_margins(self.z_cache, self.zd if self._tpend else None, self._tpend,
                                      None if with_offsets else self.o, n)
            z = self.z_cache[:n].clone()
            if self._tpend:
                z.add_(self.zd[:n], alpha=self._tpend)
            if not with_offsets:
                z.sub_(self.o[:n].to(torch.float64))
            return z
        alloc = torch.empty if getattr(self, "_masked", None) is None else torch.zeros   # skipped rows stay 0
        z = alloc(max(self.n_rows, 1), dtype=torch.float64, device=self.device)
        x = self._vec(w)
        self.fwd_all(x, FWD_MARGIN, 0, margin_shift, None, None, z_out=z, with_offset=int(with_offsets),
                     stats=False)
        return z[: self.n_rows]
