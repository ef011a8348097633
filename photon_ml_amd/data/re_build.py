"""Device-side random-effect dataset build: reservoir cap (K21), passive set and Pearson feature selection (K13).

Reference: ``photon-api/.../data/RandomEffectDataSet.scala:326-389`` (reservoir: per entity keep the
``activeDataUpperBound`` samples with the largest ``(byteswap64(reType.hashCode) ^ byteswap64(uid)).hashCode``,
re-weight by count / kept), ``:402-447`` (passive data: the remaining samples of entities with more than
``passiveDataLowerBound`` of them) and ``LocalDataSet.scala:221-280`` (Pearson correlation score per feature,
keep the ``ceil(ratio * n_e)`` features of largest |score|; the first near-constant feature scores 1, later ones 0).

Every step is a sort / segmented reduction over the whole coordinate at once (no per-entity loops), in torch on
the data's device (radix sorts and deterministic segment reductions on the GPU; the same code runs on the CPU).
Results are identical to the host implementation in ``data/random_effect.py`` (same keys, same tie order: stable
sorts in sample order, ties of |score| resolved towards the larger feature id).
"""
from __future__ import annotations

from typing import Tuple

import numpy as np
import torch

from ..constants import EPSILON

_M32 = 0xFFFFFFFF


def _bswap32(v: torch.Tensor) -> torch.Tensor:
    """Byte-reverse 32-bit values held in non-negative int64 lanes."""
    return ((v & 0xFF) << 24) | (((v >> 8) & 0xFF) << 16) | (((v >> 16) & 0xFF) << 8) | ((v >> 24) & 0xFF)


def reservoir_keys_t(type_hash: int, uids: torch.Tensor) -> torch.Tensor:
    """Java ``Long.hashCode`` of ``byteswap64(typeHash) ^ byteswap64(uid)`` (int64 tensor of signed 32-bit
    values), computed on 32-bit halves so no int64 shift ever overflows."""
    t = int(type_hash) & 0xFFFFFFFFFFFFFFFF
    t_lo, t_hi = t & _M32, (t >> 32) & _M32
    u = uids.to(torch.int64)
    u_lo, u_hi = u & _M32, (u >> 32) & _M32
    bt_hi, bt_lo = int.from_bytes(t_lo.to_bytes(4, "big"), "little"), int.from_bytes(t_hi.to_bytes(4, "big"),
                                                                                     "little")
    x_hi = _bswap32(u_lo) ^ bt_hi          # high word of byteswap64(uid) is byteswap32(low word of uid)
    x_lo = _bswap32(u_hi) ^ bt_lo
    h = x_hi ^ x_lo
    return torch.where(h >= (1 << 31), h - (1 << 32), h)


def reservoir_active_rows(ent: torch.Tensor, rows: torch.Tensor, keys: torch.Tensor, cap: int,
                          n_ent: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """(sorted active rows, per-entity weight multiplier count / kept) of a reservoir cap ``cap``."""
    e = ent[rows]
    desc = (_M32 - (keys + (1 << 31)))                       # key descending as an unsigned ascending key
    order = torch.sort(e * (1 << 32) + desc, stable=True).indices
    e_sorted = e[order]
    start = torch.searchsorted(e_sorted, e_sorted, right=False)
    rank = torch.arange(e_sorted.numel(), device=e.device) - start
    active = torch.sort(rows[order][rank < cap]).values
    counts = torch.bincount(e, minlength=n_ent).to(torch.float64)
    kept = torch.clamp(counts, max=float(cap))
    mult = torch.where(kept > 0, counts / torch.clamp(kept, min=1.0), torch.ones_like(counts))
    return active, mult


def passive_rows(ent: torch.Tensor, rows: torch.Tensor, active: torch.Tensor, n_rows: int, n_ent: int,
                 lower_bound: int) -> torch.Tensor:
    """Rows of ``rows`` that are not active, of entities with more than ``lower_bound`` such rows (sorted)."""
    is_active = torch.zeros(n_rows, dtype=torch.bool, device=rows.device)
    is_active[active] = True
    cand = rows[~is_active[rows]]
    pcount = torch.bincount(ent[cand], minlength=n_ent)
    return cand[pcount[ent[cand]] > lower_bound]


def pearson_keep_entries(row: torch.Tensor, col: torch.Tensor, val: torch.Tensor, row_ent: torch.Tensor,
                         y: torch.Tensor, n_rows_of_ent: torch.Tensor, ratio: float) -> torch.Tensor:
    """Boolean mask over the entries (``row``, ``col``, ``val``; rows local to the active set, ``row_ent`` =
    entity of each active row, ``y`` = response of each active row): entries of features that survive the
    per-entity Pearson selection. All entities at once: one sort of the (entity, feature) pairs and segment sums."""
    dev = val.device
    n_ent = n_rows_of_ent.numel()
    if val.numel() == 0:
        return torch.ones(0, dtype=torch.bool, device=dev)
    f64 = torch.float64
    e = row_ent[row]
    D = int(col.max()) + 1
    pair = e * D + col
    order = torch.sort(pair, stable=True).indices           # entries grouped by (entity, feature), row order inside
    ps = pair[order]
    first = torch.ones_like(ps, dtype=torch.bool)
    first[1:] = ps[1:] != ps[:-1]
    seg_id = torch.cumsum(first.to(torch.int64), 0) - 1     # pair index of each sorted entry
    n_pairs = int(seg_id[-1]) + 1
    lengths = torch.bincount(seg_id, minlength=n_pairs)
    v = val[order].to(f64)
    yr = y[row[order]].to(f64)
    seg = lambda t: torch.segment_reduce(t, "sum", lengths=lengths, unsafe=True)
    s1, s2, sxy = seg(v), seg(v * v), seg(v * yr)
    pair_key = ps[first]
    pe, pf = pair_key // D, pair_key % D
    # per-entity response sums over the entity's rows (sorted segment sums: deterministic, no float atomics)
    ro = torch.sort(row_ent, stable=True).indices
    ys = y.to(f64)[ro]
    rlen = torch.bincount(row_ent, minlength=n_ent)
    ly = torch.segment_reduce(ys, "sum", lengths=rlen, unsafe=True)
    ly2 = torch.segment_reduce(ys * ys, "sum", lengths=rlen, unsafe=True)
    n = n_rows_of_ent.to(f64)[pe]
    num = n * sxy - s1 * ly[pe]
    std = torch.sqrt(torch.abs(n * s2 - s1 * s1))
    den = std * torch.sqrt(torch.clamp(n * ly2[pe] - ly[pe] ** 2, min=0.0))
    score = num / (den + EPSILON)
    const = std < EPSILON
    # the first near-constant feature of an entity (lowest id: pairs are sorted) scores 1, later ones 0
    cidx = torch.nonzero(const).squeeze(1)
    first_const = torch.zeros_like(const)
    if cidx.numel():
        ce = pe[cidx]
        head = torch.ones_like(ce, dtype=torch.bool)
        head[1:] = ce[1:] != ce[:-1]
        first_const[cidx[head]] = True
    score = torch.where(const, torch.where(first_const, torch.ones_like(score), torch.zeros_like(score)), score)
    # per entity: keep the ceil(ratio * n_e) features of largest |score| (ties: larger feature id wins), or all
    k = torch.ceil(ratio * n_rows_of_ent.to(f64)).to(torch.int64)     # same float expression as math.ceil(ratio * n)
    n_feat = torch.bincount(pe, minlength=n_ent)
    a = torch.abs(score)
    o1 = torch.sort(a, stable=True).indices                 # |score| ascending, feature ascending inside ties
    o2 = o1[torch.sort(pe[o1], stable=True).indices]         # then grouped by entity
    pe2 = pe[o2]
    seg_end = torch.searchsorted(pe2, pe2, right=True)
    from_end = seg_end - torch.arange(pe2.numel(), device=dev) - 1
    keep_pair = torch.zeros(n_pairs, dtype=torch.bool, device=dev)
    keep_pair[o2] = (from_end < k[pe2]) | (k[pe2] >= n_feat[pe2])
    keep_sorted = keep_pair[seg_id]
    keep = torch.empty_like(keep_sorted)
    keep[order] = keep_sorted
    return keep

