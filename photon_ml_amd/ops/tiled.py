"""Tiled ("TL") sparse layout for the gather-coalesced HIP kernels (``glm_kernels.hip``, section TILED LAYOUT).

One row chunk of a feature shard is stored twice:

* forward copy — ROW BLOCKS of ``2^rbits`` consecutive rows; inside a block the entries are sorted by
  (column, row) and packed into one uint32 ``(col << rbits) | local_row``. Block table: ``{row_lo, nrows, e_lo,
  e_hi}``. ``rbits = min(10, 32 - bits(D))``.
* transpose copy — COLUMN TILES of ``2^cbits`` columns; inside a tile entries are sorted by (row, column) and
  packed as ``(local_row << cbits) | (col & (2^cbits - 1))``; a tile is cut into work items of at most
  ``item_entries`` entries. Item table: ``{tile, e_lo, e_hi, part}`` with ``part = -1`` for single-item tiles
  and a partial-row index otherwise; split tiles are combined in item order by a two-level fixed-order
  reduction (units of ``COMBINE_SEG`` partial rows, then the units of a tile) — deterministic.
  ``cbits = min(10, 32 - bits(chunk_rows))``.

NARROW SECTION (``PML_TL_NARROW``, default on with the interleaved layout): a unit's sorted entries are cut into
groups of 256 (one kernel round); a full group whose gather keys span fewer than 64 values (hot columns in the
forward copy, dense rows in the transpose copy: about half of the entries at the bench shape) is moved to the
unit's narrow section and stored with a 16-bit pack ``((key - base) << bits) | slot`` and one int32 ``base`` per
round (``base + 63 < len(x)``). The kernel reads such a round's key window with one coalesced load and picks the
values with cross-lane permutes (``tl_stream_narrow``): 4 B/entry of stream instead of 6 (bf16) and a third of the
gather instructions. Unit tables gain ``{n_lo, n_hi}`` (the unit's narrow rounds); a unit's narrow rounds are
processed before its remaining (wide) entries, both in sorted order.

Both copies are stored LANE-INTERLEAVED by default (``il``; ``PML_TL_IL=0`` keeps the plain order): every work
unit (forward block / transpose item) starts on a 256-entry round boundary and is zero-padded to whole rounds,
and inside a round the 16-B quad of lane L holds the unit's sorted entries L, L+64, L+128, L+192, so each gather
instruction of the kernels reads 64 consecutive sorted entries (``tl_stream_il`` in ``glm_kernels.hip``). Padding
costs < 0.5 % of the stream at the bench shapes.

The builders run with torch ops on the data's device (GPU sort for the 100M-entry bench chunks, CPU in tests).
Values keep the shard precision (bf16 / fp32 / fp64). Both copies cost 4 B + sizeof(value) per entry, the same
as the segmented-stream CSR/CSC pair they replace. Shapes the packing cannot represent (``D > 2^27`` or chunks
of more than 2^27 rows) fall back to the segmented-stream layout (:mod:`photon_ml_amd.ops.device`).
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from .native import TLFwdDesc, TLTDesc

TL_MAXBITS = 12          # kernel limit: 4096 rows per block / columns per tile (fp32 LDS: 4 waves x 16 KB)
TL_MAXBITS_F64 = 11      # fp64 LDS accumulators: 4 waves x 2048 x 8 B = 64 KB
TL_MINBITS = 5
DEFAULT_RBITS = int(os.environ.get("PML_TL_RBITS", 10))
DEFAULT_CBITS = int(os.environ.get("PML_TL_CBITS", 10))
DEFAULT_ITEM_ENTRIES = 1 << 18  # 125M rows (profiles/bench_knob_sweep.md): 64K 40.41, 128K 38.71-39.10, 256K 38.43-38.51, 512K 38.58, 1M 38.63 ms/step
_PAD = 8                 # kernels read 4-entry quads; pad so that the last quad stays in bounds
COMBINE_SEG = 16         # minimum partial rows summed per level-1 combine work-group


# XCD-aware item order of the shard-wide transpose (PML_TL_XCD=8 turns it on). Work-groups are dispatched
# round-robin over the 8 XCDs by blockIdx, each XCD has its own 4 MB L2, and an item gathers the per-row vector of
# ITS chunk (1M rows x 4 B): interleaving 8 streams (chunks c = k mod 8 in stream k) makes the blocks that share
# an XCD walk one chunk at a time. Pure scheduling (bitwise-identical results) -- but MEASURED SLOWER on the
# headline bench (40.0-40.1 vs 39.2 ms/step, profiles/bench_xcd_order_ab.md), so the default is the plain
# chunk-major order, in which all XCDs share the few in-flight chunks.
XCD_GROUPS = int(os.environ.get("PML_TL_XCD", "0"))


def xcd_order(chunk_of_item: np.ndarray, groups: int) -> np.ndarray:
    """Permutation of items (chunk-major input order kept inside each stream) such that position b holds an
    item of stream b % groups while every stream has items left."""
    stream = np.asarray(chunk_of_item) % groups
    lists = [np.flatnonzero(stream == k) for k in range(groups)]
    longest = max(len(l) for l in lists)
    grid = np.full((longest, groups), -1, dtype=np.int64)
    for k, l in enumerate(lists):
        grid[: len(l), k] = l
    order = grid.reshape(-1)
    return order[order >= 0]


def combine_seg(k: int) -> int:
    """Partial rows per level-1 combine unit of a tile split into ``k`` items: ~sqrt(k) (at least COMBINE_SEG), so
    neither level loops over more than ~sqrt(k) rows per thread. A hot tile of a 125M-row shard has ~47K items:
    fixed 16-row units left its level-2 sum a 2.9K-long serial chain per thread (1 ms per pass, measured)."""
    return max(COMBINE_SEG, int(math.ceil(math.sqrt(k))))
IL_ROUND = 256           # entries per wave-round of the kernels (64 lanes x 4-entry quads)
TL_VEC = 4               # entries per lane per round
INTERLEAVE = int(os.environ.get("PML_TL_IL", "1"))
NARROW = int(os.environ.get("PML_TL_NARROW", "1"))
NARROW_W = 64            # key window loaded per narrow round (one wave64 load)
WIDE_BASE = int(os.environ.get("PML_TL_WIDE_BASE", "1"))   # per-round key bases for wide shards (TLFwdChunk)


def narrow_width(sbits: int) -> int:
    """Largest key span of a narrow round: the 16-bit pack holds (key - base) in 16 - sbits bits."""
    return min(NARROW_W, 1 << max(16 - sbits, 0))


def _bits(n: int) -> int:
    return max(1, int(n - 1).bit_length())


def _cap(want: int, f64: bool) -> int:
    return min(want, TL_MAXBITS_F64 if f64 else TL_MAXBITS)


# fp64 shards over wide feature spaces use 2048-row forward blocks: an fp64 coefficient gather covers half the
# columns per cache line of an fp32 one, so the denser keys of a bigger block pay there (game5pl fp64 fixed effect:
# 54.4 -> 52.2 ms per coordinate update; the bf16 shards are faster with 1024-row blocks: 32.2 vs 33.2 ms;
# profiles/tl_tile_knobs_r4.md). PML_TL_RBITS overrides.
F64_WIDE_RBITS = 11


def default_rbits(dim: int, f64: bool) -> int:
    if f64 and dim >= (1 << 16) and "PML_TL_RBITS" not in os.environ:
        return F64_WIDE_RBITS
    return DEFAULT_RBITS


def fwd_bits(dim: int, f64: bool = False, want: Optional[int] = None) -> Optional[int]:
    r = min(_cap(default_rbits(dim, f64) if want is None else want, f64), 32 - _bits(dim))
    return r if r >= TL_MINBITS else None


def t_bits(chunk_rows: int, f64: bool = False, want: Optional[int] = None) -> Optional[int]:
    c = min(_cap(DEFAULT_CBITS if want is None else want, f64), 32 - _bits(chunk_rows))
    return c if c >= TL_MINBITS else None


# Sparse shards: when a 1024-column tile of a row chunk holds fewer than this many entries on average, the transpose
# copies use 2048-column tiles and 128K-entry items instead (measured on the game5pl fixed-effect shard, 25M rows x
# 30 non-zeros over 1M features, ~31K entries per tile and chunk: FE coordinate 34.65 -> 32.83 ms; the headline
# shard, ~102K entries per tile and chunk, is faster with the defaults: 37.88 vs 38.12 ms/step;
# profiles/tl_tile_knobs_r4.md). PML_TL_CBITS / PML_TL_ITEM_ENTRIES override.
SPARSE_TILE_ENTRIES = 1 << 16


def shard_t_config(nnz: int, n_rows: int, dim: int, chunk_rows: int):
    """``(cbits, item_entries)`` for the transpose copies of a whole shard (one choice for every chunk: the
    shard-wide transpose needs one tile width); ``(None, None)`` = the defaults."""
    if "PML_TL_CBITS" in os.environ or "PML_TL_ITEM_ENTRIES" in os.environ or n_rows <= 0 or dim < (1 << 16):
        return None, None                      # (small feature spaces keep the defaults: a few tiles at most)
    per_tile = (nnz / n_rows) * min(chunk_rows, n_rows) / math.ceil(dim / 1024)
    if per_tile < SPARSE_TILE_ENTRIES:
        return 11, 1 << 17
    return None, None


def tl_supported(dim: int, chunk_rows: int) -> bool:
    return fwd_bits(dim) is not None and t_bits(chunk_rows) is not None


def _to_u32_bits(x64: torch.Tensor) -> torch.Tensor:
    """int64 values in [0, 2^32) -> int32 tensor with the same low 32 bits (the kernels read uint32)."""
    return torch.where(x64 >= (1 << 31), x64 - (1 << 32), x64).to(torch.int32)


def _pad(t: torch.Tensor) -> torch.Tensor:
    return torch.cat([t, torch.zeros(_PAD, dtype=t.dtype, device=t.device)]).contiguous()


def il_phys(e_lo: torch.Tensor, n: torch.Tensor) -> torch.Tensor:
    """Physical positions of the logical entries of units starting at ``e_lo`` (round-aligned) with ``n``
    entries each, in unit order: logical j of a unit lives at e_lo + 256*(j//256) + 4*(j%64) + (j%256)//64."""
    e_lo = e_lo.to(torch.int64)
    n = n.to(torch.int64)
    tot = int(n.sum())
    unit = torch.repeat_interleave(torch.arange(n.numel(), device=n.device), n)
    j = torch.arange(tot, device=n.device) - (torch.cumsum(n, 0) - n)[unit]
    t = j & (IL_ROUND - 1)
    return e_lo[unit] + (j - t) + ((t & 63) << 2) + (t >> 6)


def _interleave(pack: torch.Tensor, val: torch.Tensor, n: torch.Tensor):
    """Lane-interleave sorted streams whose units are consecutive runs of ``n`` entries. Returns the padded
    streams and the new (round-aligned) unit starts."""
    n = n.to(torch.int64)
    padded = (n + IL_ROUND - 1) // IL_ROUND * IL_ROUND
    new_lo = torch.cumsum(padded, 0) - padded
    total = int(padded.sum()) + _PAD
    phys = il_phys(new_lo, n)
    p = torch.zeros(total, dtype=pack.dtype, device=pack.device)
    v = torch.zeros(total, dtype=val.dtype, device=val.device)
    p[phys] = pack
    v[phys] = val
    return p, v, new_lo


def _empty_narrow(val: torch.Tensor):
    dev = val.device
    return (torch.zeros(IL_ROUND, dtype=torch.int16, device=dev), torch.zeros(IL_ROUND, dtype=val.dtype, device=dev),
            torch.zeros(1, dtype=torch.int32, device=dev))


def split_narrow(pack: torch.Tensor, val: torch.Tensor, n: torch.Tensor, sbits: int, xlen: int, enable: bool = True):
    """Move the narrow rounds of every unit out of sorted, unit-contiguous streams.

    ``pack`` (int64, low 32 bits = the packed entry ``key << sbits | slot``) and ``val`` hold units of ``n[u]``
    consecutive entries, each unit sorted by key. Returns ``(wide_pack, wide_val, wide_n, npack, nval, nbase,
    nrounds)``: the remaining entries per unit (same order), the interleaved 16-bit narrow stream (int16 bit
    patterns), its values, one base per narrow round and the number of narrow rounds per unit."""
    dev = pack.device
    n = n.to(torch.int64)
    U = n.numel()
    gcount = n // IL_ROUND
    W = narrow_width(sbits)
    ok = enable and NARROW and W >= 16 and xlen >= NARROW_W and int(gcount.sum()) > 0
    if not ok:
        z = torch.zeros(U, dtype=torch.int64, device=dev)
        return (pack, val, n, *_empty_narrow(val), z)
    starts = torch.cumsum(n, 0) - n
    gu = torch.repeat_interleave(torch.arange(U, device=dev), gcount)
    gi = torch.arange(gu.numel(), device=dev) - (torch.cumsum(gcount, 0) - gcount)[gu]
    gs = starts[gu] + IL_ROUND * gi
    key = pack >> sbits
    first, last = key[gs], key[gs + IL_ROUND - 1]
    base = torch.clamp(first, max=xlen - NARROW_W)        # the 64-wide window load stays inside x
    nar = (last - base) < W
    gs_n, base = gs[nar], base[nar]
    idx = gs_n[:, None] + torch.arange(IL_ROUND, device=dev)[None, :]
    p16 = ((key[idx] - base[:, None]) << sbits) | (pack[idx] & ((1 << sbits) - 1))
    # interleave: logical t = 64 k + L of a round lives at 4 L + k
    il = lambda t: t.reshape(-1, TL_VEC, 64).transpose(1, 2).reshape(-1)
    npack = il(torch.where(p16 >= 32768, p16 - 65536, p16).to(torch.int16)).contiguous()
    nval = il(val[idx]).contiguous()
    nbase = base.to(torch.int32).contiguous()
    # narrow rounds per unit: gu is non-decreasing (units' rounds are consecutive), so a prefix sum of the flags read
    # at the unit boundaries (torch.bincount on these long runs of one bin serialised its atomics)
    cs = torch.zeros(nar.numel() + 1, dtype=torch.int64, device=dev)
    torch.cumsum(nar.to(torch.int64), 0, out=cs[1:])
    ge = torch.cumsum(gcount, 0)
    nrounds = cs[ge] - cs[ge - gcount]
    keep = torch.ones(pack.numel(), dtype=torch.bool, device=dev)
    keep[idx.reshape(-1)] = False
    del idx, p16
    return pack[keep], val[keep], n - IL_ROUND * nrounds, npack, nval, nbase, nrounds



def narrow_logical(npack: torch.Tensor, nval: torch.Tensor, nbase: torch.Tensor, r_lo, r_hi, sbits: int):
    """(pack32 as int64, val) of narrow rounds [r_lo, r_hi) in logical order."""
    r = torch.arange(int(r_lo), int(r_hi), device=npack.device)
    if not r.numel():
        return torch.zeros(0, dtype=torch.int64, device=npack.device), nval[:0]
    ph = (r[:, None] * IL_ROUND + torch.arange(IL_ROUND, device=npack.device)[None, :]).reshape(-1, 64, TL_VEC)
    ph = ph.transpose(1, 2).reshape(-1)          # physical position of logical entry t of each round
    p16 = npack[ph].to(torch.int64) & 0xFFFF
    base = nbase[r].to(torch.int64).repeat_interleave(IL_ROUND)
    return (((p16 >> sbits) + base) << sbits) | (p16 & ((1 << sbits) - 1)), nval[ph]


class _NarrowMixin:
    """Narrow-section bookkeeping shared by the forward and transpose chunks (``table`` columns 4, 5 hold the
    per-unit narrow round range [n_lo, n_hi); the wide window is columns ``_ew``)."""

    wbase = None          # forward copies only: int32 key base per physical wide round (see TLFwdChunk)

    def _set_narrow(self, npack, nval, nbase):
        from .native import TLNarrow
        self.npack, self.nval, self.nbase = npack, nval, nbase
        self.nar = TLNarrow(npack.data_ptr(), nval.data_ptr(), nbase.data_ptr(),
                            None if self.wbase is None else self.wbase.data_ptr())

    @property
    def n_narrow_rounds(self) -> int:
        t = self._table()
        return int((t[:, 5] - t[:, 4]).sum()) if t.shape[0] else 0

    def unit_counts(self) -> torch.Tensor:
        t = self._table().to(torch.int64)
        lo, hi = self._ew
        return (t[:, hi] - t[:, lo]) + IL_ROUND * (t[:, 5] - t[:, 4])

    def narrow_window(self, r_lo: int, r_hi: int):
        return narrow_logical(self.npack, self.nval, self.nbase, r_lo, r_hi, self._sbits)

    def _logical_all(self, wide_pack, wide_val):
        """Units in table order; inside a unit its narrow entries, then its wide entries."""
        t = self._table().to(torch.int64)
        dev = wide_pack.device
        lo, hi = self._ew
        nn = IL_ROUND * (t[:, 5] - t[:, 4])
        nw = t[:, hi] - t[:, lo]
        if int(nn.sum()) == 0:
            return wide_pack, wide_val
        npk, nvl = narrow_logical(self.npack, self.nval, self.nbase, 0, int(t[:, 5].max()), self._sbits)
        # narrow rounds of a unit are consecutive and in unit order -> gather them unit by unit
        U = t.shape[0]
        nu = torch.repeat_interleave(torch.arange(U, device=dev), nn.to(dev))
        nj = torch.arange(int(nn.sum()), device=dev) - (torch.cumsum(nn, 0) - nn).to(dev)[nu]
        npos = t[:, 4].to(dev)[nu] * IL_ROUND + nj
        wu = torch.repeat_interleave(torch.arange(U, device=dev), nw.to(dev))
        unit = torch.cat([nu, wu])
        order = torch.sort(unit, stable=True).indices
        wp = wide_pack.to(torch.int64) & 0xFFFFFFFF if wide_pack.dtype == torch.int32 else wide_pack.to(torch.int64)
        pk = torch.cat([npk[npos], wp])[order]
        vl = torch.cat([nvl[npos], wide_val])[order]
        return pk, vl


class TLFwdChunk(_NarrowMixin):
    """Forward copy of one row chunk (``m`` rows)."""

    kind = "tl"

    def __init__(self, rowptr: torch.Tensor, col: torch.Tensor, val: torch.Tensor, dim: int,
                 rbits: Optional[int] = None, il: Optional[int] = None):
        dev = val.device
        self.il = INTERLEAVE if il is None else int(il)
        rowptr = rowptr.to(dev, torch.int64)
        col = col.to(dev, torch.int64)
        m = rowptr.numel() - 1
        f64 = val.dtype == torch.float64
        self.rbits = fwd_bits(dim, f64, rbits)
        if self.rbits is None:
            raise ValueError(f"tiled forward layout cannot pack dim={dim}")
        # wide shards: (col << rbits) would overflow 32 bits at the wanted block size -> keys relative to one base
        # per wide round (the full block size instead of 2^(32 - bits(D)) rows; see tl_stream_ring)
        want = _cap(default_rbits(dim, f64) if rbits is None else rbits, f64)
        use_base = bool(self.il) and WIDE_BASE and want > self.rbits
        if use_base:
            self.rbits = want
        R = 1 << self.rbits
        kbits = _bits(dim) + self.rbits                       # bits of (col << rbits) | row
        nnz = col.numel()
        rows = torch.repeat_interleave(torch.arange(m, device=dev), rowptr[1:] - rowptr[:-1]) if nnz else \
            torch.zeros(0, dtype=torch.int64, device=dev)
        pack = (col << self.rbits) | (rows & (R - 1))
        key = ((rows >> self.rbits) << kbits) | pack
        key, perm = torch.sort(key, stable=True)
        nblk = (m + R - 1) // R
        b = torch.arange(nblk, device=dev)
        lo = b * R
        hi = torch.clamp(lo + R, max=m)
        e_lo, e_hi = rowptr[lo], rowptr[hi]
        self._sbits, self._ew = self.rbits, (2, 3)
        n_lo = n_hi = torch.zeros(nblk, dtype=torch.int64, device=dev)
        if self.il:
            wp, wv, wn, npk, nvl, nbs, nr = split_narrow(key & ((1 << kbits) - 1), val[perm], e_hi - e_lo,
                                                         self.rbits, dim)
            del key, perm
            if use_base:
                wp = self._rebase(wp, wn)
                if wp is None:      # a wide round spans more keys than 32 - rbits bits: plain packs, fewer rows
                    del wv, npk, nvl, nbs
                    self.__init__(rowptr, col, val, dim, fwd_bits(dim, f64, rbits), il)
                    return
            self.pack, self.val, e_lo = _interleave(_to_u32_bits(wp), wv, wn)
            e_hi = e_lo + wn
            n_hi = torch.cumsum(nr, 0)
            n_lo = n_hi - nr
            del wp, wv
        else:
            self.pack = _pad(_to_u32_bits(key & ((1 << kbits) - 1)))
            self.val = _pad(val[perm].contiguous())
            npk, nvl, nbs = _empty_narrow(val)
            del key, perm
        del rows
        self._set_narrow(npk, nvl, nbs)
        self.blk = torch.stack([lo, hi - lo, e_lo, e_hi, n_lo, n_hi], 1).to(torch.int32).contiguous()
        self.nblk, self.m, self.nnz = nblk, m, nnz
        self.desc = TLFwdDesc(self.blk.data_ptr(), nblk, self.rbits, self.pack.data_ptr(), self.val.data_ptr(),
                              self.il, self.nar)

    def _rebase(self, wp: torch.Tensor, wn: torch.Tensor) -> Optional[torch.Tensor]:
        """Wide packs (int64 ``(key << rbits) | slot``, units of ``wn`` sorted entries) relative to the first key of
        their round of the interleaved layout; sets ``self.wbase`` (int32 per physical round). None when some
        round's key span does not fit 32 - rbits bits."""
        dev = wp.device
        n = wn.to(torch.int64)
        tot = int(n.sum())
        padded = (n + IL_ROUND - 1) // IL_ROUND * IL_ROUND
        nrounds = int(padded.sum()) // IL_ROUND
        wbase = torch.zeros(nrounds + 1, dtype=torch.int64, device=dev)
        if tot:
            unit = torch.repeat_interleave(torch.arange(n.numel(), device=dev), n, output_size=tot)
            j = torch.arange(tot, device=dev) - (torch.cumsum(n, 0) - n)[unit]
            rid = ((torch.cumsum(padded, 0) - padded)[unit] + j) // IL_ROUND     # same rounds as _interleave
            del unit
            key = wp >> self.rbits
            first = (j % IL_ROUND) == 0
            del j
            wbase[rid[first]] = key[first]
            rel = key - wbase[rid]
            del rid, key, first
            if int(rel.max()) >= 1 << (32 - self.rbits):
                return None
            wp = (rel << self.rbits) | (wp & ((1 << self.rbits) - 1))
        self.wbase = wbase.to(torch.int32).contiguous()
        return wp

    @property
    def nstats(self) -> int:
        return self.nblk

    parts_needed = 0

    def _table(self):
        return self.blk

    def nbytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in (self.blk, self.pack, self.val, self.npack, self.nval,
                                                           self.nbase) + (() if self.wbase is None else (self.wbase,)))

    def logical(self):
        """(pack, val) of the non-zeros in unit order (per block: its narrow entries, then its wide entries, each
        sorted by column), whatever the storage order; packs as non-negative int64 ``(col << rbits) | row``."""
        if not self.il:
            return self.pack[: self.nnz].to(torch.int64) & 0xFFFFFFFF, self.val[: self.nnz]
        ph = il_phys(self.blk[:, 2], self.blk[:, 3] - self.blk[:, 2])
        wp = self.pack[ph].to(torch.int64) & 0xFFFFFFFF
        if self.wbase is not None:
            wp = ((self.wbase[ph // IL_ROUND].to(torch.int64) + (wp >> self.rbits)) << self.rbits) | (
                wp & ((1 << self.rbits) - 1))
        return self._logical_all(wp, self.val[ph])

    # host emulation of the kernel arithmetic (tests / CPU fallback)
    def emulate_matvec(self, x: torch.Tensor) -> torch.Tensor:
        pk, vl = self.logical()
        p = pk.to(torch.int64)
        col = p >> self.rbits
        blk_of_entry = torch.repeat_interleave(torch.arange(self.nblk, device=p.device), self.unit_counts())
        row = (blk_of_entry << self.rbits) + (p & ((1 << self.rbits) - 1))
        z = torch.zeros(self.m, dtype=torch.float64, device=p.device)
        return z.index_add_(0, row, vl.to(torch.float64) * x.to(torch.float64)[col])


class TLTChunk(_NarrowMixin):
    """Transpose copy of one row chunk."""

    kind = "tl"

    def __init__(self, rowptr: torch.Tensor, col: torch.Tensor, val: torch.Tensor, dim: int, chunk_rows: int,
                 cbits: Optional[int] = None, item_entries: Optional[int] = None, il: Optional[int] = None):
        self.il = INTERLEAVE if il is None else int(il)
        if item_entries is None:
            item_entries = int(os.environ.get("PML_TL_ITEM_ENTRIES", DEFAULT_ITEM_ENTRIES))
        dev = val.device
        rowptr = rowptr.to(dev, torch.int64)
        col = col.to(dev, torch.int64)
        m = rowptr.numel() - 1
        self.cbits = t_bits(max(chunk_rows, m), val.dtype == torch.float64, cbits)
        if self.cbits is None:
            raise ValueError(f"tiled transpose layout cannot pack chunk_rows={chunk_rows}")
        C = 1 << self.cbits
        nnz = col.numel()
        rows = torch.repeat_interleave(torch.arange(m, device=dev), rowptr[1:] - rowptr[:-1]) if nnz else \
            torch.zeros(0, dtype=torch.int64, device=dev)
        tile = col >> self.cbits
        pack = (rows << self.cbits) | (col & (C - 1))
        key = (tile << 32) | pack
        del rows, pack
        key, perm = torch.sort(key, stable=True)
        del tile
        ntiles = (dim + C - 1) // C
        # entries per tile from the sorted keys (tile = key >> 32): binary search, no atomics
        tptr = torch.searchsorted(key >> 32, torch.arange(ntiles + 1, device=dev)).cpu().numpy().astype(np.int64)
        counts = np.diff(tptr)
        pack = _to_u32_bits(key & 0xFFFFFFFF)
        val = val[perm]
        del key, perm
        nz = np.nonzero(counts)[0]
        n_it = np.maximum(1, -(-counts[nz] // item_entries))
        # items of every non-empty tile, vectorised: item i of a tile of k items covers [a + (b-a) i / k, ...)
        it_tile = np.repeat(nz, n_it)
        it_i = np.arange(len(it_tile)) - np.repeat(np.cumsum(n_it) - n_it, n_it)
        it_k = np.repeat(n_it, n_it)
        a, b = tptr[it_tile], tptr[it_tile + 1]
        lo, hi = a + (b - a) * it_i // it_k, a + (b - a) * (it_i + 1) // it_k
        split = it_k > 1
        part_of = np.full(len(it_tile), -1, np.int64)
        part_of[split] = np.arange(int(split.sum()))
        # level-1 combine units of ~sqrt(k) consecutive partial rows per split tile (combine_seg)
        km = n_it[n_it > 1]
        plo = np.cumsum(km) - km
        sg = np.maximum(COMBINE_SEG, np.ceil(np.sqrt(km)).astype(np.int64)) if len(km) else km
        nu = -(-km // sg)
        u_mt = np.repeat(np.arange(len(km)), nu)
        u_first = np.repeat(plo, nu) + np.repeat(sg, nu) * (np.arange(int(nu.sum())) - np.repeat(np.cumsum(nu) - nu, nu))
        u_last = np.minimum(u_first + np.repeat(sg, nu), np.repeat(plo + km, nu))
        cu = np.column_stack([u_mt, u_first, u_last]) if len(km) else np.zeros((0, 3), np.int64)
        mt_tiles = nz[n_it > 1].tolist()
        mt_ptr = np.r_[0, np.cumsum(nu)].tolist() if len(km) else [0]
        self.nitems, self.nmt, self.nparts, self.ncu = len(it_tile), len(mt_tiles), int(km.sum()), len(cu)
        items = np.column_stack([it_tile, lo, hi, part_of]).astype(np.int64).reshape(-1, 4)
        items = np.column_stack([items, np.zeros((len(items), 2), np.int64)])
        self._sbits, self._ew = self.cbits, (1, 2)
        if self.il:
            cnt = torch.from_numpy(items[:, 2] - items[:, 1]).to(dev)
            wp, wv, wn, npk, nvl, nbs, nr = split_narrow(pack.to(torch.int64) & 0xFFFFFFFF, val, cnt, self.cbits, m)
            del pack, val
            self.pack, self.val, new_lo = _interleave(_to_u32_bits(wp), wv, wn)
            del wp, wv
            items[:, 1] = new_lo.cpu().numpy()
            items[:, 2] = items[:, 1] + wn.cpu().numpy()
            nr = nr.cpu().numpy()
            items[:, 5] = np.cumsum(nr)
            items[:, 4] = items[:, 5] - nr
        else:
            self.pack, self.val = _pad(pack), _pad(val.contiguous())
            npk, nvl, nbs = _empty_narrow(val)
            del pack, val
        self._set_narrow(npk, nvl, nbs)
        self.items = torch.tensor(items.astype(np.int32), device=dev)
        self.mt_tiles = torch.tensor(np.asarray(mt_tiles or [0], dtype=np.int32), device=dev)
        self.mt_ptr = torch.tensor(np.asarray(mt_ptr, dtype=np.int32), device=dev)
        self.cu = torch.tensor(np.asarray(cu if len(cu) else [(0, 0, 0)], dtype=np.int32).reshape(-1, 3), device=dev)
        self.m, self.nnz, self.dim = m, nnz, dim
        self.desc = TLTDesc(self.items.data_ptr(), self.nitems, self.cbits, self.pack.data_ptr(),
                            self.val.data_ptr(), self.mt_tiles.data_ptr(), self.mt_ptr.data_ptr(), self.nmt, dim,
                            self.cu.data_ptr(), self.ncu, self.nparts, self.il, self.nar)

    @property
    def parts_needed(self) -> int:
        """fp64 scratch: item partial rows followed by the level-1 combine rows."""
        return (self.nparts + self.ncu) << self.cbits

    def _table(self):
        return self.items

    def nbytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in (self.items, self.mt_tiles, self.mt_ptr, self.cu, self.pack,
                                                           self.val, self.npack, self.nval, self.nbase))

    def window(self, e_lo: int, e_hi: int):
        """(pack, val) of one item's wide window in sorted order."""
        if not self.il:
            return self.pack[e_lo:e_hi], self.val[e_lo:e_hi]
        ph = il_phys(torch.tensor([e_lo]), torch.tensor([e_hi - e_lo])).to(self.pack.device)
        return self.pack[ph], self.val[ph]

    def logical(self):
        if not self.il:
            return self.pack[: self.nnz], self.val[: self.nnz]
        ph = il_phys(self.items[:, 1], self.items[:, 2] - self.items[:, 1])
        return self._logical_all(self.pack[ph], self.val[ph])

    def emulate_rmatvec(self, r: torch.Tensor, square: bool = False) -> torch.Tensor:
        pk, vl = self.logical()
        p = pk.to(torch.int64) & 0xFFFFFFFF
        row = p >> self.cbits
        tile_of_entry = torch.repeat_interleave(self.items[:, 0].to(torch.int64), self.unit_counts())
        col = (tile_of_entry << self.cbits) + (p & ((1 << self.cbits) - 1))
        v = vl.to(torch.float64)
        if square:
            v = v * v
        g = torch.zeros(self.dim, dtype=torch.float64, device=p.device)
        return g.index_add_(0, col, v * r.to(torch.float64)[row])


class TLTMulti:
    """Shard-wide transpose over every row chunk in one launch (``tl_t_multi_kernel``).

    Items of all chunks keep their launch order (chunk, item); each carries its chunk (stream pointers), its row
    base (offset into the shard-length row vector) and a partial-row slot. Tiles hit by more than one item in the
    whole shard are combined by the same two-level fixed-order combine as a single chunk's split tiles, so the
    result is deterministic and independent of chunk scheduling. Requires one ``cbits`` for all chunks and
    column windows (if any) that start on tile boundaries (``tile_offsets``).
    """

    def __init__(self, chunks: Sequence["TLTChunk"], row_starts: Sequence[int], dim: int,
                 tile_range: Optional[Tuple[int, int]] = None, tile_offsets: Optional[Sequence[int]] = None):
        """``tile_range`` = [t0, t1): only the items of those column tiles (a gradient BUCKET: columns
        [t0 * C, t1 * C) are final after this launch + its combine, so their all-reduce can start).
        ``tile_offsets``: per chunk, the global tile of its local tile 0 (chunks stored in tile-aligned column
        windows); tiles that several chunks' items share are combined like split tiles."""
        from .native import TLTMultiDesc
        dev = chunks[0].pack.device
        self.cbits = chunks[0].cbits
        self.il = chunks[0].il
        if any(ch.il != self.il for ch in chunks):
            raise ValueError("TLTMulti: chunks mix interleaved and plain streams")
        its = []
        for c, ch in enumerate(chunks):
            it = ch.items[: ch.nitems].cpu().numpy().astype(np.int64).reshape(-1, 6)
            toff = 0 if tile_offsets is None else int(tile_offsets[c])
            its.append(np.column_stack([np.full(len(it), c), it[:, 0] + toff, it[:, 1], it[:, 2],
                                        np.full(len(it), row_starts[c]), it[:, 4], it[:, 5]]))
        it = np.concatenate(its) if its else np.zeros((0, 7), np.int64)
        src_all = np.arange(len(it))
        if tile_range is not None:
            in_range = (it[:, 1] >= tile_range[0]) & (it[:, 1] < tile_range[1])
            it = it[in_range]
        n = len(it)
        tile = it[:, 1]
        order = np.lexsort((np.arange(n), tile))          # grouped by tile, (chunk, item) order inside
        ts = tile[order]
        starts = np.flatnonzero(np.r_[True, ts[1:] != ts[:-1]]) if n else np.zeros(0, np.int64)
        k = np.diff(np.r_[starts, n])                    # items per tile (shard-wide)
        multi_tile = np.repeat(k > 1, k)
        part = np.full(n, -1, np.int64)
        part[order[multi_tile]] = np.arange(int(multi_tile.sum()))
        # level-1 units of <= COMBINE_SEG consecutive partial rows per split tile
        km = k[k > 1]
        plo = np.cumsum(km) - km
        sg = np.maximum(COMBINE_SEG, np.ceil(np.sqrt(km)).astype(np.int64)) if len(km) else km
        nu = -(-km // sg)
        u_tile = np.repeat(np.arange(len(km)), nu)
        u_first = np.repeat(plo, nu) + np.repeat(sg, nu) * (np.arange(int(nu.sum())) - np.repeat(np.cumsum(nu) - nu, nu))
        u_last = np.minimum(u_first + np.repeat(sg, nu), np.repeat(plo + km, nu))
        self.nitems, self.nparts, self.ncu, self.nmt = n, int(km.sum()), int(nu.sum()), len(km)
        rows = np.column_stack([it[:, 0], it[:, 1], it[:, 2], it[:, 3], part, it[:, 4], it[:, 5],
                                it[:, 6]]).astype(np.int32)
        src = src_all if tile_range is None else src_all[in_range]
        if XCD_GROUPS > 1 and n > XCD_GROUPS:
            xo = xcd_order(it[:, 0], XCD_GROUPS)
            rows, src = rows[xo], src[xo]
        self._src = torch.from_numpy(src.astype(np.int64)).to(dev)   # row -> index into the chunks' concatenated items
        self.items = torch.tensor(rows.reshape(-1, 8), device=dev)
        self.mt_tiles = torch.tensor(np.r_[ts[starts][k > 1], 0].astype(np.int32)[: max(self.nmt, 1)], device=dev)
        self.mt_ptr = torch.tensor(np.r_[0, np.cumsum(nu)].astype(np.int32), device=dev)
        self.cu = torch.tensor(np.column_stack([u_tile, u_first, u_last]).astype(np.int32).reshape(-1, 3)
                               if self.ncu else np.zeros((1, 3), np.int32), device=dev)
        self.ptrs = stream_ptr_table(chunks, dev)
        self._chunks = list(chunks)  # keep the streams alive
        self.desc = TLTMultiDesc(self.items.data_ptr(), n, self.cbits, self.ptrs.data_ptr(),
                                 self.mt_tiles.data_ptr(), self.mt_ptr.data_ptr(), self.nmt, dim,
                                 self.cu.data_ptr(), self.ncu, self.nparts, self.il)

    @property
    def parts_needed(self) -> int:
        return (self.nparts + self.ncu) << self.cbits

    def restreamed(self, chunks: Sequence["TLTChunk"]) -> "TLTMulti":
        """The same launch over other streams of the SAME units (row-sampled copies, ``RowCompaction``): every
        row's stream window and narrow range come from ``chunks``' item tables (one device gather), tiles,
        partial-row slots and combine tables are shared. No host work beyond the pointer table."""
        import copy
        from .native import TLTMultiDesc
        dev = self.items.device
        cat = torch.cat([ch.items[: ch.nitems].to(torch.int64) for ch in chunks]) if chunks else None
        rows = self.items.to(torch.int64).clone()
        if self.nitems:
            sel = cat[self._src]
            rows[:, 2:4] = sel[:, 1:3]
            rows[:, 6:8] = sel[:, 4:6]
        new = copy.copy(self)
        new.items = rows.to(torch.int32).contiguous()
        new.ptrs = stream_ptr_table(chunks, dev)
        new._chunks = list(chunks)
        d = self.desc
        new.desc = TLTMultiDesc(new.items.data_ptr(), d.nitems, d.cbits, new.ptrs.data_ptr(), d.mt_tiles, d.mt_ptr,
                                d.nmt, d.dim, d.cu, d.ncu, d.nparts_total, d.il)
        return new

    def emulate_rmatvec(self, r: torch.Tensor, square: bool = False) -> torch.Tensor:
        """Host emulation of the launch + combine (item partial rows, direct tiles, two-level combine)."""
        C = 1 << self.cbits
        dim = self.desc.dim
        ntiles = (dim + C - 1) // C
        G = torch.zeros(ntiles * C, dtype=torch.float64)
        parts = torch.zeros((max(self.nparts, 1), C), dtype=torch.float64)
        r = r.to(torch.float64).cpu()
        for c, tile, e_lo, e_hi, part, rb, n_lo, n_hi in self.items.cpu().tolist():
            ch = self._chunks[c]
            pk, vl = ch.window(e_lo, e_hi)
            npk, nvl = ch.narrow_window(n_lo, n_hi)
            p = torch.cat([npk.cpu(), pk.to(torch.int64).cpu() & 0xFFFFFFFF])
            v = torch.cat([nvl.cpu(), vl.cpu()]).to(torch.float64)
            if square:
                v = v * v
            acc = torch.zeros(C, dtype=torch.float64).index_add_(0, p & (C - 1), v * r[rb + (p >> self.cbits)])
            if part < 0:
                G[tile * C:(tile + 1) * C] += acc
            else:
                parts[part] = acc
        cu = self.cu.cpu().tolist()
        l1 = [parts[a:b].sum(0) for _, a, b in cu[: self.ncu]]
        mp = self.mt_ptr.cpu().tolist()
        for t, tile in enumerate(self.mt_tiles.cpu().tolist()[: self.nmt]):
            s = torch.zeros(C, dtype=torch.float64)
            for u in range(mp[t], mp[t + 1]):
                s += l1[u]
            G[tile * C:(tile + 1) * C] += s
        return G[:dim]


def stream_ptr_table(chunks, device) -> torch.Tensor:
    """Per-chunk stream pointers of the shard-wide kernels: {pack, val, narrow pack, narrow val, narrow base,
    wide-round bases (0: absolute keys)}."""
    wb = lambda ch: 0 if getattr(ch, "wbase", None) is None else ch.wbase.data_ptr()
    return torch.tensor([[ch.pack.data_ptr(), ch.val.data_ptr(), ch.npack.data_ptr(), ch.nval.data_ptr(),
                          ch.nbase.data_ptr(), wb(ch)] for ch in chunks], dtype=torch.int64,
                        device=device).reshape(-1)


# ---- row-sampled copies (K20 down-sampling work saving: DeviceGLMData.row_sampled) ---------------------------
CMP_SEG = 8              # rounds of one unit per compaction segment (tl_compact_kernel, one wave each)


def _cmp_segments(ch, narrow: bool):
    """Segment table of a chunk's units (cached per ``narrow``): int32 {unit, round_lo, round_hi} per segment, a
    unit's rounds numbered narrow first, then wide ([nn, nn + wide rounds)); ``narrow=False``: the wide rounds
    only. Plus each segment's unit, the unit's first segment (int64) and the chunk's narrow entry count."""
    cache = ch.__dict__.setdefault("_cmp_seg", {})
    if cache.get(narrow) is not None:
        return cache[narrow]
    t = ch._table().to(torch.int64)
    dev = t.device
    lo, hi = ch._ew
    nn = t[:, 5] - t[:, 4]
    R = (t[:, hi] - t[:, lo] + IL_ROUND - 1) // IL_ROUND + (nn if narrow else 0)
    ns = (R + CMP_SEG - 1) // CMP_SEG
    S = int(ns.sum())
    su = torch.repeat_interleave(torch.arange(t.shape[0], device=dev), ns, output_size=S)
    first = (torch.cumsum(ns, 0) - ns)[su]
    r_lo = (torch.arange(S, device=dev) - first) * CMP_SEG
    r_hi = torch.minimum(r_lo + CMP_SEG, R[su])
    if not narrow:
        r_lo, r_hi = r_lo + nn[su], r_hi + nn[su]
    seg = torch.stack([su, r_lo, r_hi], 1).to(torch.int32).contiguous()
    cache[narrow] = (seg, su, first, S, IL_ROUND * int(nn.sum()))
    return cache[narrow]


class RowCompaction:
    """Row-sampled copy of one interleaved tiled chunk (forward or transpose copy) by ``tl_compact_kernel``:
    the constructor queues the counting pass and the device-side scans (``total`` / ``kept`` stay on the device so
    that all chunks of a shard need ONE host sync), :meth:`finish` allocates the compacted streams, queues the
    writing pass and returns the new chunk. Every unit keeps its table slot (row block / transpose item, split-tile
    partial rows and combine tables unchanged).

    ``filter_narrow=False`` (most rows kept): only the WIDE entries are filtered and the narrow section is shared
    with the full chunk as is — a filtered narrow round no longer spans < 64 keys, and a wide round costs 4.4x a
    narrow round of texture-address time (``profiles/pmc_tl_multi_125M_r3.md``), so converting them made a
    half-kept shard as slow as the full one; the dropped rows' narrow entries still run (weight 0: their per-row
    coefficient is 0, their margins are never used). ``True`` (few rows kept, below ~80/352 of a round): the
    narrow entries are filtered too and the copy is all wide rounds."""

    def __init__(self, ch, keep: torch.Tensor, forward: bool, filter_narrow: bool = False):
        from .native import CmpArgs, check, require_game_lib, stream_handle
        if not ch.il:
            raise ValueError("row-sampled copies need the interleaved layout")
        self.ch, self.keep, self.forward = ch, keep, forward
        dev = ch.pack.device
        self.filter_narrow = bool(filter_narrow)
        seg, su, first, S, self.n_narrow = _cmp_segments(ch, self.filter_narrow)
        table = ch._table()
        lo, hi = ch._ew
        self.seg_cnt = torch.zeros(max(S, 1), dtype=torch.int32, device=dev)
        self._keep_alive = (seg, table, keep)
        self.args = CmpArgs(table.data_ptr(), lo, 0 if forward else -1, seg.data_ptr(), S, ch._sbits,
                            0 if forward else 1, ch.pack.data_ptr(), ch.val.data_ptr(), ch.npack.data_ptr(),
                            ch.nval.data_ptr(), ch.nbase.data_ptr(), keep.data_ptr(), self.seg_cnt.data_ptr(),
                            None, None, None, None)
        self.lib, self.stream = require_game_lib(), stream_handle(dev)
        self.vbytes = ch.val.element_size()
        if S:
            check(self.lib.pml_tl_compact(0, self.vbytes, ctypes.byref(self.args), self.stream), "tl_compact count")
        cnt = self.seg_cnt[:S].to(torch.int64)
        U = table.shape[0]
        self.unit_cnt = torch.zeros(U, dtype=torch.int64, device=dev).index_add_(0, su, cnt)
        padded = (self.unit_cnt + IL_ROUND - 1) // IL_ROUND * IL_ROUND
        self.unit_lo = (torch.cumsum(padded, 0) - padded).contiguous()
        excl = torch.cumsum(cnt, 0) - cnt
        self.seg_first = (excl - excl[first]).contiguous() if S else excl
        self.total, self.kept = padded.sum(), self.unit_cnt.sum()

    def finish(self, total: int, kept: int):
        import copy
        from .native import TLFwdDesc, TLTDesc, check
        ch = self.ch
        dev = ch.pack.device
        opack = torch.zeros(total + _PAD, dtype=torch.int32, device=dev)
        oval = torch.zeros(total + _PAD, dtype=ch.val.dtype, device=dev)
        a = self.args
        a.seg_first, a.unit_lo = self.seg_first.data_ptr(), self.unit_lo.data_ptr()
        a.opack, a.oval = opack.data_ptr(), oval.data_ptr()
        if a.nseg:
            check(self.lib.pml_tl_compact(1, self.vbytes, ctypes.byref(a), self.stream), "tl_compact write")
        lo, hi = ch._ew
        table = ch._table().to(torch.int64).clone()
        table[:, lo] = self.unit_lo
        table[:, hi] = self.unit_lo + self.unit_cnt
        if self.filter_narrow:
            table[:, 4:6] = 0
        table = table.to(torch.int32).contiguous()
        nc = copy.copy(ch)               # shares the narrow streams (npack / nval / nbase, table columns 4, 5)
        nc._cmp_seg = {}
        nc.pack, nc.val = opack, oval
        if self.filter_narrow:
            nc._set_narrow(*_empty_narrow(oval))
            nc.nnz = kept
        else:
            nc.nnz = kept + self.n_narrow
        if self.forward:
            nc.blk = table
            nc.desc = TLFwdDesc(table.data_ptr(), nc.nblk, nc.rbits, opack.data_ptr(), oval.data_ptr(), 1, nc.nar)
        else:
            nc.items = table
            nc.desc = TLTDesc(table.data_ptr(), nc.nitems, nc.cbits, opack.data_ptr(), oval.data_ptr(),
                              nc.mt_tiles.data_ptr(), nc.mt_ptr.data_ptr(), nc.nmt, nc.dim, nc.cu.data_ptr(), nc.ncu,
                              nc.nparts, 1, nc.nar)
        return nc
