"""Random-effect datasets: entity grouping, active/passive split, reservoir cap, Pearson feature selection,
projection, and the bucketed dense layout consumed by the batched solvers.

Reference: ``photon-api/.../data/RandomEffectDataSet.scala`` (active data via groupByKey or the reservoir cap
``326-389``; passive data ``402-447``; feature selection ``458-476``), ``LocalDataSet.scala`` (Pearson scores
``221-280``), ``RandomEffectDataSetPartitioner.scala`` (entity -> partition bin packing) and
``data/CoordinateDataConfiguration.scala`` (``RandomEffectDataConfiguration``).

MI355X-first layout: entities are sorted by (active rows, projected dim) and packed into BUCKETS of similar
shape; each bucket is one dense zero-padded tensor ``X [B, n_max, d_max]`` resident on the device plus the
sample index of every slot, so the per-update residual routing (C11) is a single gather of the N-length offset
vector and the per-entity solves are batched (``optimization/batched.py``). Multi-GPU entity sharding uses the
same greedy least-loaded bin packing as the reference partitioner (``parallel/sharding.py``).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np
import scipy.sparse as sp
import torch

from ..constants import EPSILON
from ..projector.projectors import (IndexMapProjection, ProjectorKind, ProjectorType, gaussian_projection_matrix)
from .game_data import GameData
from .matrix import DeviceCSR, LabeledData
from ..utils.timing import phase


@dataclass
class RandomEffectDataConfiguration:
    random_effect_type: str
    feature_shard_id: str
    min_partitions: int = 1
    active_data_upper_bound: Optional[int] = None
    passive_data_lower_bound: Optional[int] = None
    features_to_samples_ratio: Optional[float] = None
    projector_type: ProjectorType = field(default_factory=lambda: ProjectorType())

    def __post_init__(self):
        self.projector_type = ProjectorType.parse(self.projector_type)
        if self.active_data_upper_bound is not None and self.active_data_upper_bound <= 0:
            raise ValueError("active data upper bound must be positive")
        if self.passive_data_lower_bound is not None and self.passive_data_lower_bound < 0:
            raise ValueError("passive data lower bound must be non-negative")
        if self.features_to_samples_ratio is not None and self.features_to_samples_ratio <= 0:
            raise ValueError("features to samples ratio must be positive")


@dataclass
class FixedEffectDataConfiguration:
    feature_shard_id: str
    min_partitions: int = 1


# ----------------------------------------------------------------------------------------------------------------
# Reservoir key (RandomEffectDataSet.scala:361-367): (byteswap64(reType.hashCode) ^ byteswap64(uid)).hashCode()
def java_string_hash(s: str) -> int:
    h = 0
    for ch in s:
        h = (31 * h + ord(ch)) & 0xFFFFFFFF
    return h - (1 << 32) if h >= (1 << 31) else h


def _byteswap64(v: np.ndarray) -> np.ndarray:
    return v.astype(np.uint64).byteswap()


def reservoir_keys(re_type: str, uids: np.ndarray) -> np.ndarray:
    t = np.array([java_string_hash(re_type)], dtype=np.int64).astype(np.uint64)
    x = _byteswap64(t) ^ _byteswap64(uids.astype(np.int64).astype(np.uint64))
    h = (x ^ (x >> np.uint64(32))) & np.uint64(0xFFFFFFFF)
    return h.astype(np.int64) - ((h >= (1 << 31)).astype(np.int64) << 32)


def pearson_scores(xe: sp.csr_matrix, y: np.ndarray) -> dict:
    """LocalDataSet.computePearsonCorrelationScore for one entity's rows (first near-constant feature -> 1)."""
    n = xe.shape[0]
    coo = xe.tocoo()
    feats = np.unique(coo.col)
    s1 = np.bincount(coo.col, weights=coo.data, minlength=xe.shape[1])
    s2 = np.bincount(coo.col, weights=coo.data ** 2, minlength=xe.shape[1])
    sxy = np.bincount(coo.col, weights=coo.data * y[coo.row], minlength=xe.shape[1])
    ly, ly2 = y.sum(), (y * y).sum()
    out = {}
    intercept_added = False
    for j in feats:
        num = n * sxy[j] - s1[j] * ly
        std = math.sqrt(abs(n * s2[j] - s1[j] * s1[j]))
        den = std * math.sqrt(max(n * ly2 - ly * ly, 0.0))
        if std < EPSILON:
            score = 0.0 if intercept_added else 1.0
            intercept_added = True
        else:
            score = num / (den + EPSILON)
        out[int(j)] = score
    return out


@dataclass
class SegmentSubset:
    """Block-diagonal sub-problem over some entities of a segmented coordinate (``entity_subset``)."""
    seg: object               # SegmentedGLMData over the subset
    rows: torch.Tensor        # positions of its rows in the parent's (entity-sorted) row order
    cols: torch.Tensor        # positions of its coefficients in the parent's coefficient vector
    entities: torch.Tensor    # parent entity index of each subset entity


@dataclass
class Bucket:
    entities: np.ndarray      # entity indices in this bucket [B]
    rows: torch.Tensor        # [B, n] global sample index of each slot, -1 for padding
    X: torch.Tensor           # [B, n, d] projected features
    y: torch.Tensor           # [B, n]
    w: torch.Tensor           # [B, n] (0 on padding, x reservoir multiplier)
    d_local: np.ndarray       # projected dim per entity


def sorted_factors(codes: np.ndarray, table) -> Optional[tuple]:
    """``np.unique(ids.astype(str), return_inverse=True)`` from a factorisation ``ids = table[codes]``: the sort
    runs over the distinct values only. None when two distinct values print to the same string (mixed id types),
    which only the per-row path merges the same way."""
    us = np.asarray(table, dtype=object).astype(str)
    order = np.argsort(us, kind="stable")
    u = us[order]
    if len(u) > 1 and bool((u[1:] == u[:-1]).any()):
        return None
    rank = np.empty(len(order), dtype=np.int64)
    rank[order] = np.arange(len(order), dtype=np.int64)
    return u, rank[np.asarray(codes, dtype=np.int64)]


def factorize_ids(ids: np.ndarray) -> Optional[tuple]:
    """:func:`sorted_factors` of a per-row object array through a hash factorisation (4x faster than np.unique of
    the strings at 10M rows); None for missing values (pandas would print them as "nan", np.unique as "None")."""
    import pandas as pd
    codes, uniq = pd.factorize(ids, sort=False, use_na_sentinel=False)
    if bool(pd.isna(uniq).any()):
        return None
    return sorted_factors(codes, uniq)



# PML_LAZY_SEG_LAYOUT=0 builds the random-effect coordinate's pass layout eagerly with the dataset (as before round 6)
LAZY_SEG_LAYOUT = os.environ.get("PML_LAZY_SEG_LAYOUT", "1") != "0"


class LazyGLMData:
    """A GLM pass backend built on first use: any attribute access builds it (once) and delegates. ``built`` tells
    whether that has happened (without building)."""

    def __init__(self, build):
        self._build = build
        self._obj = None

    @property
    def built(self) -> bool:
        return self._obj is not None

    def _get(self):
        if self._obj is None:
            self._obj = self._build()
            self._build = None             # drops the closure's references to the CSR inputs
        return self._obj

    def __getattr__(self, name):
        if name.startswith("__") or name in ("_build", "_obj"):
            raise AttributeError(name)
        return getattr(self._get(), name)

class RandomEffectDataset:
    """Active/passive data of one random-effect coordinate, projected and bucketed."""

    def __init__(self, data: GameData, config: RandomEffectDataConfiguration, device="cpu",
                 dtype=torch.float64, bucket_elems: int = 1 << 24, entity_subset: Optional[np.ndarray] = None,
                 layout: str = "auto"):
        """``layout``: ``dense`` = size buckets of padded ``[B, n, d]`` problems (batched GEMMs); ``segmented`` =
        one block-diagonal sparse GLM over all entities (INDEX_MAP projection only; the GLM kernels do the
        products, no padding). ``auto`` = segmented for INDEX_MAP on a GPU, dense otherwise."""
        self.config = config
        self.device = torch.device(device)
        self.dtype = dtype
        re_type, shard_id = config.random_effect_type, config.feature_shard_id
        x = data.shard(shard_id)
        # device copy of the shard started by GameData.prefetch_shard (used by the segmented device build below when
        # every row is active; taken here in any case so an unused copy is released)
        prefetched = data.take_prefetched(shard_id, x) if hasattr(data, "take_prefetched") else None
        if isinstance(x, DeviceCSR) and not (
                self.device.type == "cuda" and layout in ("auto", "segmented")
                and config.projector_type.kind == ProjectorKind.INDEX_MAP and config.features_to_samples_ratio is None):
            x = x.to_scipy()      # device-resident rows (entity-sharded routing) on a host-only build path
        self.dim = x.shape[1]
        ids = data.id_tags[re_type]
        with phase("RE dataset: entity ids"):
            fac = (getattr(data, "id_factors", None) or {}).get(re_type)
            got = None
            if fac is not None and fac[2] is ids and len(fac[0]) == len(ids):
                got = sorted_factors(fac[0], fac[1])          # the reader's codes: no per-row string work
            elif ids.dtype == object and len(ids):
                got = factorize_ids(ids)
            ids_s = ids.astype(str) if got is None and ids.dtype == object else ids
            if got is not None:
                self.entity_ids, ent = got
            elif self.device.type == "cuda" and np.issubdtype(ids_s.dtype, np.integer) and len(ids_s):
                # integer entity ids: sorted unique + inverse on the device (np.unique: 1.3 s at 25M rows)
                u, inv = torch.unique(torch.from_numpy(np.ascontiguousarray(ids_s)).to(self.device), sorted=True,
                                      return_inverse=True)
                self.entity_ids, ent = u.cpu().numpy().astype(ids_s.dtype, copy=False), inv.cpu().numpy()
            else:
                self.entity_ids, ent = np.unique(ids_s, return_inverse=True)
        n_ent = len(self.entity_ids)
        n = data.n_rows
        self.n_rows = n
        self.sample_entity = ent.astype(np.int64)
        rows = np.arange(n, dtype=np.int64)
        if entity_subset is not None:  # entity sharding across ranks: keep only owned entities
            own = np.zeros(n_ent, dtype=bool)
            own[entity_subset] = True
            rows = rows[own[ent]]
        # ---- active data (optionally reservoir-capped)
        weight_mult = np.ones(n)
        counts = np.bincount(ent[rows], minlength=n_ent)
        cap = config.active_data_upper_bound
        # K21 / K13 on the device (data/re_build.py: whole-coordinate sorts + segment reductions)
        mode = os.environ.get("PML_RE_DEVICE_BUILD", "1")   # "0" host numpy, "force" torch ops even on the CPU
        self.device_build = (self.device.type == "cuda" and mode != "0") or mode == "force"
        if self.device_build:
            from . import re_build
            dev = self.device
            ent_t = torch.from_numpy(ent.astype(np.int64)).to(dev)
            rows_t = torch.from_numpy(rows).to(dev)
        if cap is not None and self.device_build:
            keys_t = re_build.reservoir_keys_t(java_string_hash(re_type),
                                               torch.from_numpy(np.asarray(data.uids[rows], dtype=np.int64)).to(dev))
            act_t, mult_t = re_build.reservoir_active_rows(ent_t, rows_t, keys_t, cap, n_ent)
            active_rows = act_t.cpu().numpy()
            weight_mult[active_rows] = mult_t.cpu().numpy()[ent[active_rows]]
        elif cap is not None:
            key = reservoir_keys(re_type, data.uids[rows])
            order = np.lexsort((-key, ent[rows]))  # by entity, key descending
            r_sorted = rows[order]
            e_sorted = ent[r_sorted]
            start = np.searchsorted(e_sorted, e_sorted, side="left")
            rank = np.arange(len(r_sorted)) - start
            keep = rank < cap
            active_rows = np.sort(r_sorted[keep])
            kept = np.minimum(counts, cap)
            mult = np.where(kept > 0, counts / np.maximum(kept, 1), 1.0)
            weight_mult[active_rows] = mult[ent[active_rows]]
        else:
            active_rows = rows
        self.active_rows = active_rows
        self.weight_mult = weight_mult
        # ---- passive data
        passive_rows = np.zeros(0, dtype=np.int64)
        if config.passive_data_lower_bound is not None and self.device_build:
            passive_rows = re_build.passive_rows(ent_t, rows_t, torch.from_numpy(active_rows).to(dev), n, n_ent,
                                                 config.passive_data_lower_bound).cpu().numpy()
        elif config.passive_data_lower_bound is not None:
            is_active = np.zeros(n, dtype=bool)
            is_active[active_rows] = True
            cand = rows[~is_active[rows]]
            pcount = np.bincount(ent[cand], minlength=n_ent)
            passive_rows = cand[pcount[ent[cand]] > config.passive_data_lower_bound]
        self.passive_rows = passive_rows
        self.score_mask = np.zeros(n, dtype=bool)
        self.score_mask[active_rows] = True
        self.score_mask[passive_rows] = True
        # ---- feature selection (Pearson) on active rows
        xa = x if len(active_rows) == n else x[active_rows]  # no copy when every row is active
        ea = ent[active_rows]
        self.feature_keep = None
        if config.features_to_samples_ratio is not None:
            xa = self._pearson_filter(xa, ea, data.response[active_rows], config.features_to_samples_ratio)
        self.x_active = xa
        pt = config.projector_type
        self.projector_type = pt
        n_act = np.bincount(ea, minlength=n_ent)
        self.n_active = n_act
        if layout == "auto":
            layout = "segmented" if (pt.kind == ProjectorKind.INDEX_MAP and self.device.type == "cuda") else "dense"
        if layout == "segmented" and pt.kind != ProjectorKind.INDEX_MAP:
            raise ValueError("the segmented random-effect layout needs the INDEX_MAP projector")
        self.layout = layout
        self.buckets = []
        self.seg = None
        wts = weight_mult * data.weights
        if layout == "segmented" and self.device.type == "cuda":
            # GPU build: projection + entity-sorted block-diagonal layout computed on the device
            with phase("RE dataset: segmented layout"):
                self._make_segmented_device(x, xa, ea, ent, active_rows, passive_rows, data.response, wts, n_ent,
                                            prefetched=prefetched if xa is x else None)
            self.d_local = self.projection.local_dims()
            return
        # ---- projection
        if pt.kind == ProjectorKind.INDEX_MAP:
            coo = xa.tocoo()
            e_all = ea[coo.row]
            f_all = coo.col
            if len(passive_rows):
                cp = x[passive_rows].tocoo()
                e_all = np.concatenate([e_all, ent[passive_rows][cp.row]])
                f_all = np.concatenate([f_all, cp.col])
            self.projection = IndexMapProjection.build(e_all, f_all, n_ent, self.dim)
            d_local = self.projection.local_dims()
        elif pt.kind == ProjectorKind.RANDOM:
            self.matrix = gaussian_projection_matrix(pt.projected_dim, self.dim, keep_intercept=True)
            d_local = np.full(n_ent, self.matrix.shape[0], dtype=np.int64)
        else:
            d_local = np.full(n_ent, self.dim, dtype=np.int64)
        self.d_local = d_local
        # ---- buckets (dense) or one block-diagonal problem (segmented)
        if layout == "segmented":
            self._make_segmented(xa, ea, active_rows, data.response, wts, n_ent)
        else:
            self.buckets = self._make_buckets(xa, ea, active_rows, data.response, wts, n_act, d_local,
                                              bucket_elems)

    # ------------------------------------------------------------------
    def _pearson_filter(self, xa: sp.csr_matrix, ea: np.ndarray, y: np.ndarray, ratio: float) -> sp.csr_matrix:
        if getattr(self, "device_build", False):
            return self._pearson_filter_device(xa, ea, y, ratio)
        xa = xa.tocsr()
        order = np.argsort(ea, kind="stable")
        keep_mask_rows = []
        out_rows, out_cols, out_vals = [], [], []
        starts = np.searchsorted(ea[order], np.arange(ea.max() + 2 if len(ea) else 1))
        xa_coo = xa.tocoo()
        keep_entry = np.ones(xa.nnz, dtype=bool)
        row_ent = ea
        # per entity: compute scores over its rows, keep top-k features
        by_ent = {}
        for e in np.unique(ea):
            r = order[starts[e]:starts[e + 1]]
            xe = xa[r]
            k = int(math.ceil(ratio * len(r)))
            n_feat = len(np.unique(xe.indices))
            if k >= n_feat:
                continue
            scores = pearson_scores(xe, y[r])
            ranked = sorted(scores.items(), key=lambda kv: abs(kv[1]))
            keep = {f for f, _ in ranked[-k:]}
            by_ent[e] = keep
        if not by_ent:
            return xa
        ent_of_entry = row_ent[xa_coo.row]
        for e, keep in by_ent.items():
            m = ent_of_entry == e
            keep_entry[m] = np.isin(xa_coo.col[m], np.fromiter(keep, dtype=np.int64))
        return sp.csr_matrix((xa_coo.data[keep_entry], (xa_coo.row[keep_entry], xa_coo.col[keep_entry])),
                             shape=xa.shape)

    def _pearson_filter_device(self, xa: sp.csr_matrix, ea: np.ndarray, y: np.ndarray, ratio: float):
        """K13 for every entity at once on the device (data/re_build.pearson_keep_entries)."""
        from .re_build import pearson_keep_entries
        dev = self.device
        coo = xa.tocoo()
        n_ent = int(ea.max()) + 1 if len(ea) else 0
        keep = pearson_keep_entries(torch.from_numpy(coo.row.astype(np.int64)).to(dev),
                                    torch.from_numpy(coo.col.astype(np.int64)).to(dev),
                                    torch.from_numpy(coo.data.astype(np.float64)).to(dev),
                                    torch.from_numpy(ea.astype(np.int64)).to(dev),
                                    torch.from_numpy(np.asarray(y, dtype=np.float64)).to(dev),
                                    torch.bincount(torch.from_numpy(ea.astype(np.int64)).to(dev), minlength=n_ent),
                                    ratio).cpu().numpy()
        return sp.csr_matrix((coo.data[keep], (coo.row[keep], coo.col[keep])), shape=xa.shape)

    def _matrix_t(self, device) -> torch.Tensor:
        """P^T [D x k] of the random projection as a device fp64 tensor (uploaded once)."""
        cache = self.__dict__.setdefault("_mt_cache", {})
        if str(device) not in cache:
            cache[str(device)] = torch.from_numpy(np.ascontiguousarray(self.matrix.T, dtype=np.float64)).to(device)
        return cache[str(device)]

    def _project_rows(self, xr: sp.csr_matrix, er: np.ndarray):
        """Return (row_idx, local_col, value) triplets of rows ``xr`` of entities ``er`` in projected space."""
        pt = self.projector_type
        if pt.kind == ProjectorKind.INDEX_MAP:
            coo = xr.tocoo()
            lc = self.projection.local_index(er[coo.row], coo.col)
            ok = lc >= 0
            return coo.row[ok], lc[ok], coo.data[ok]
        if pt.kind == ProjectorKind.RANDOM:
            if self.device.type == "cuda":
                # K15 forward map on the device (spmm_rows_kernel): one wave per row over the k projected dims
                from ..ops.native import spmm_rows
                dense = spmm_rows(xr, self._matrix_t(self.device)).cpu().numpy()
            else:
                dense = np.asarray(xr @ self.matrix.T)
            r, c = np.nonzero(dense)
            return r, c, dense[r, c]
        coo = xr.tocoo()
        return coo.row, coo.col, coo.data

    def _make_buckets(self, xa, ea, active_rows, y, wts, n_act, d_local, budget) -> List[Bucket]:
        n_ent = len(n_act)
        ents = np.nonzero(n_act > 0)[0]
        order = ents[np.lexsort((d_local[ents], n_act[ents]))]
        buckets_e: List[List[int]] = []
        cur: List[int] = []
        n0 = d0 = nm = dm = 0
        for e in order:
            ne, de = int(n_act[e]), max(int(d_local[e]), 1)
            if cur:
                nm2, dm2 = max(nm, ne), max(dm, de)
                if ((len(cur) + 1) * nm2 * dm2 > budget) or nm2 > 2 * n0 + 8 or dm2 > 2 * d0 + 8:
                    buckets_e.append(cur)
                    cur = []
            if not cur:
                n0, d0, nm, dm = ne, de, ne, de
            nm, dm = max(nm, ne), max(dm, de)
            cur.append(e)
        if cur:
            buckets_e.append(cur)
        # rows of each entity (active), in sample order
        ord_rows = np.argsort(ea, kind="stable")
        starts = np.zeros(n_ent + 1, dtype=np.int64)
        starts[1:] = np.cumsum(n_act)
        out = []
        for be in buckets_e:
            be = np.asarray(be, dtype=np.int64)
            B = len(be)
            nmax = int(n_act[be].max())
            dmax = max(int(d_local[be].max()), 1)
            loc_rows = np.concatenate([ord_rows[starts[e]:starts[e + 1]] for e in be])  # into active arrays
            slot_b = np.repeat(np.arange(B), n_act[be])
            slot_r = np.concatenate([np.arange(n_act[e]) for e in be])
            xr = xa[loc_rows]
            rr, cc, vv = self._project_rows(xr, ea[loc_rows])
            X = np.zeros((B, nmax, dmax))
            X[slot_b[rr], slot_r[rr], cc] = vv
            rows = np.full((B, nmax), -1, dtype=np.int64)
            rows[slot_b, slot_r] = active_rows[loc_rows]
            Y = np.zeros((B, nmax))
            Y[slot_b, slot_r] = y[active_rows[loc_rows]]
            W = np.zeros((B, nmax))
            W[slot_b, slot_r] = wts[active_rows[loc_rows]]
            dev, dt = self.device, self.dtype
            out.append(Bucket(be, torch.from_numpy(rows).to(dev), torch.from_numpy(X).to(dev, dt),
                              torch.from_numpy(Y).to(dev, dt), torch.from_numpy(W).to(dev, dt), d_local[be]))
        return out

    def _make_segmented(self, xa, ea, active_rows, y, wts, n_ent):
        from ..ops.backend import make_glm_data
        from ..optimization.batched import SegmentedGLMData
        order = np.argsort(ea, kind="stable")        # active rows grouped by entity (sample order inside)
        xs = xa[order].tocoo()
        e_row = ea[order]
        pos = self.projection.local_index(e_row[xs.row], xs.col) + self.projection.ptr[e_row[xs.row]]
        d_total = int(self.projection.ptr[-1])
        x_seg = sp.csr_matrix((xs.data, (xs.row, pos)), shape=(len(order), max(d_total, 1)))
        rows = active_rows[order]
        yy = np.asarray(y, dtype=np.float64)[rows]
        ww = np.asarray(wts, dtype=np.float64)[rows]
        glm = make_glm_data(LabeledData(x_seg, yy, np.zeros(len(rows)), ww), self.device, "f64", col_windows=True)
        dev = glm.device
        self._seg_csr = (torch.from_numpy(x_seg.indptr.astype(np.int64)), torch.from_numpy(
            x_seg.indices.astype(np.int64)), torch.from_numpy(x_seg.data.astype(np.float64)))
        col_entity = np.repeat(np.arange(n_ent, dtype=np.int64), np.diff(self.projection.ptr))
        self.seg_rows = torch.from_numpy(rows).to(dev)
        self.projection_keys_t = torch.from_numpy(self.projection.keys).to(dev)
        self.col_entity_t = torch.from_numpy(col_entity).to(dev)
        self.seg = SegmentedGLMData(glm, torch.from_numpy(e_row.astype(np.int64)).to(dev),
                                    self.col_entity_t, n_ent,
                                    torch.from_numpy(yy).to(dev), torch.from_numpy(ww).to(dev),
                                    torch.zeros(len(rows), dtype=torch.float64, device=dev))
        self.d_total = d_total

    def _make_segmented_device(self, x, xa, ea, ent, active_rows, passive_rows, y, wts, n_ent, prefetched=None):
        """Device build of the block-diagonal problem (K14 on the GPU): rows sorted by entity (stable), the
        INDEX_MAP projection = sorted unique ``entity * D + feature`` keys of the active (+ passive) non-zeros,
        each non-zero's block column = its key's rank; then the tiled layout is built from the device CSR."""
        from ..ops.device import DeviceGLMData
        from ..optimization.batched import SegmentedGLMData
        dev, D = self.device, self.dim
        xa = xa.tocsr()
        with phase("RE segmented: upload"):
            if isinstance(xa, DeviceCSR):        # routed rows already on the device: no host copy
                ip = xa.indptr.to(dev)
                x_ind, x_val = xa.indices.to(dev), xa.data.to(dev)
            elif prefetched is not None:         # copied by GameData.prefetch_shard while the GPU built other layouts
                ip, x_ind, x_val = prefetched
            else:
                ip = torch.from_numpy(xa.indptr.astype(np.int64)).to(dev)
                x_ind, x_val = torch.from_numpy(xa.indices).to(dev), torch.from_numpy(xa.data).to(dev, torch.float64)
        sort_phase = phase("RE segmented: entity sort + projection keys")
        sort_phase.__enter__()
        ea_t = torch.from_numpy(ea.astype(np.int64)).to(dev)
        order = torch.argsort(ea_t, stable=True)
        lens = (ip[1:] - ip[:-1])[order]
        nip = torch.zeros(len(ea) + 1, dtype=torch.int64, device=dev)
        torch.cumsum(lens, 0, out=nip[1:])
        nnz = int(nip[-1])
        src = torch.repeat_interleave(ip[:-1][order] - nip[:-1], lens, output_size=nnz)
        src += torch.arange(nnz, device=dev)
        del ip
        with phase("RE keys: entity-order gather"):
            col = x_ind[src].to(torch.int64)
            val = x_val[src]
        del src, x_ind, x_val
        e_row = ea_t[order]
        key = torch.repeat_interleave(e_row, lens, output_size=nnz) * D + col
        del col, lens
        allk = key
        if len(passive_rows) and isinstance(x, DeviceCSR):
            sub = x[passive_rows]
            plen = sub.indptr[1:] - sub.indptr[:-1]
            pe = torch.from_numpy(ent[passive_rows].astype(np.int64)).to(dev)
            pk = torch.repeat_interleave(pe, plen.to(dev), output_size=sub.nnz) * D + sub.indices.to(dev, torch.int64)
            allk = torch.cat([key, pk])
        elif len(passive_rows):
            cp = x[passive_rows].tocoo()
            pk = torch.from_numpy(ent[passive_rows][cp.row].astype(np.int64) * D + cp.col.astype(np.int64))
            allk = torch.cat([key, pk.to(dev)])
        with phase("RE keys: unique"):
            ukeys = torch.unique(allk, sorted=True)
        n_keys_in = int(allk.numel())
        del allk
        # cheap integrity checks of the device build (first / last key, no more keys than entries): a corrupt
        # projection would send every later per-entity gather out of bounds on the device
        if ukeys.numel():
            lo_k, hi_k = (int(v) for v in torch.stack([ukeys[0], ukeys[-1]]).tolist())
            if lo_k < 0 or hi_k >= n_ent * D or ukeys.numel() > n_keys_in:
                raise RuntimeError(f"random-effect projection keys out of range: [{lo_k}, {hi_k}] for {n_ent} "
                                   f"entities x {D} features, {ukeys.numel()} keys from {n_keys_in} entries")
        self.projection = IndexMapProjection.from_sorted_keys(ukeys, n_ent, D)
        with phase("RE keys: entry ranks"):
            pos = torch.searchsorted(ukeys, key)
        del key
        d_total = int(ukeys.numel())
        rows_t = torch.from_numpy(active_rows.astype(np.int64)).to(dev)[order]
        yy = torch.from_numpy(np.asarray(y, dtype=np.float64)).to(dev)[rows_t]
        ww = torch.from_numpy(np.asarray(wts, dtype=np.float64)).to(dev)[rows_t]
        sort_phase.__exit__(None, None, None)
        # the block-diagonal pass layout (tiled forward / transpose tables) is built on its first use: with the fused
        # solvers (row space, per-entity primal TRON) a GAME run typically never runs a pass over the whole
        # coordinate (game5pl: 0.6 s of the 2.0 s build), and the CSR below serves the solver setup
        def build_glm(nip=nip, pos=pos, val=val, yy=yy, ww=ww, d=max(d_total, 1)):
            with phase("RE segmented: tiled layout"):
                return DeviceGLMData.from_device_csr(nip, pos, val, yy, torch.zeros_like(yy), ww, d, dev, "f64",
                                                     col_windows=True)
        glm = LazyGLMData(build_glm) if LAZY_SEG_LAYOUT else build_glm()
        self._seg_csr = (nip, pos, val)   # kept until the primal sub-problem is built (entity_subset), then freed
        self.projection_keys_t = ukeys
        self.col_entity_t = ukeys // D
        self.seg_rows = rows_t
        # rows already grouped by entity and all active (generated / pre-sorted data): the per-update offset gather
        # and score scatter through seg_rows are identities and are skipped
        self.seg_rows_identity = bool(rows_t.numel() == len(y) and (
            rows_t.numel() == 0 or bool((rows_t == torch.arange(rows_t.numel(), device=dev)).all())))
        self.seg = SegmentedGLMData(glm, e_row, self.col_entity_t, n_ent, yy, ww,
                                    torch.zeros_like(yy))
        self.d_total = d_total

    def entity_subset(self, mask: torch.Tensor) -> "SegmentSubset":
        """The block-diagonal sub-problem of the entities in ``mask`` (their rows and coefficient ranges only),
        built on the data's device from the kept CSR. Used for the primal solve of the entities NOT handled in
        their row space: its Hessian-vector passes then stream only those entities' non-zeros (with power-law
        entity sizes, ~40 % of them) instead of the whole coordinate."""
        from ..ops.backend import make_glm_data
        from ..ops.device import DeviceGLMData
        from ..optimization.batched import SegmentedGLMData
        seg = self.seg
        sip, spos, sval, row_sel, col_sel, ent_new = self.entity_csr(mask)
        dev = seg.y.device
        mask = mask.to(dev)
        B = int(mask.sum())
        d_sub = int(col_sel.numel())
        yy, ww = seg.y[row_sel], seg.w[row_sel]
        if dev.type == "cuda":
            glm = DeviceGLMData.from_device_csr(sip, spos, sval, yy, torch.zeros_like(yy), ww, max(d_sub, 1), dev,
                                                "f64", col_windows=True)
        else:
            from .matrix import LabeledData as _LD
            xs = sp.csr_matrix((sval.numpy(), spos.numpy(), sip.numpy()), shape=(row_sel.numel(), max(d_sub, 1)))
            glm = make_glm_data(_LD(xs, yy.numpy(), np.zeros(row_sel.numel()), ww.numpy()), dev, "f64",
                                col_windows=True)
        sub = SegmentedGLMData(glm, ent_new[seg.row_entity[row_sel]], ent_new[seg.col_entity[col_sel]], B, yy, ww,
                               torch.zeros_like(yy))
        return SegmentSubset(sub, row_sel, col_sel, torch.nonzero(mask).squeeze(1))

    def entity_csr(self, mask: torch.Tensor):
        """Raw block-diagonal CSR of the entities in ``mask`` (from the kept segmented CSR, on the data's device):
        ``(indptr, columns, values, row_sel, col_sel, ent_new)`` — int64 indptr over the selected rows, int64
        columns renumbered to the selected coefficients (each entity's range stays contiguous), fp64 values; the
        parent row / coefficient positions of the selection; and the parent-entity -> subset-entity numbering."""
        if getattr(self, "_seg_csr", None) is None:
            raise RuntimeError("entity_subset needs the segmented CSR (built once per dataset)")
        seg = self.seg
        nip, pos, val = self._seg_csr
        dev = seg.y.device
        mask = mask.to(dev)
        row_sel = torch.nonzero(mask[seg.row_entity]).squeeze(1)
        col_mask = mask[seg.col_entity]
        col_sel = torch.nonzero(col_mask).squeeze(1)
        newcol = torch.cumsum(col_mask.to(torch.int64), 0) - 1
        nip_d, pos_d, val_d = nip.to(dev), pos.to(dev), val.to(dev)
        lens = (nip_d[1:] - nip_d[:-1])[row_sel]
        sip = torch.zeros(row_sel.numel() + 1, dtype=torch.int64, device=dev)
        torch.cumsum(lens, 0, out=sip[1:])
        nnz = int(sip[-1])
        src = torch.repeat_interleave(nip_d[:-1][row_sel] - sip[:-1], lens, output_size=nnz) + torch.arange(
            nnz, device=dev)
        spos = newcol[pos_d[src]]
        sval = val_d[src].to(torch.float64)
        ent_new = torch.cumsum(mask.to(torch.int64), 0) - 1
        return sip, spos, sval, row_sel, col_sel, ent_new

    def entity_rows(self, mask: torch.Tensor):
        """``(row_sel, col_sel)``: parent row positions and parent coefficient positions of the entities in
        ``mask`` (each entity's rows and coefficient range stay contiguous and in order). No non-zero-sized work:
        callers gather the rows' entries themselves (``ops.native.csr_gather_rows``)."""
        seg = self.seg
        mask = mask.to(seg.y.device)
        if os.environ.get("PML_CHECK_KERNEL_INPUTS", "0") == "1":
            for name, t in (("row", seg.row_entity), ("column", seg.col_entity)):
                if t.numel() and (int(t.min()) < 0 or int(t.max()) >= mask.numel()):
                    raise RuntimeError(f"{name} entity index out of range [0, {mask.numel()})")
        return torch.nonzero(mask[seg.row_entity]).squeeze(1), torch.nonzero(mask[seg.col_entity]).squeeze(1)

    def release_csr(self):
        self._seg_csr = None

    @property
    def n_entities(self) -> int:
        return len(self.entity_ids)

    def bucket_offsets(self, bucket: Bucket, offsets: torch.Tensor) -> torch.Tensor:
        """Gather per-slot offsets (C11 residual routing): offsets is the N-length vector on the device."""
        r = bucket.rows.clamp(min=0)
        o = offsets.to(self.device, self.dtype)[r]
        return torch.where(bucket.rows >= 0, o, torch.zeros_like(o))

    def summary(self) -> str:
        d = self.d_local[self.n_active > 0]
        return (f"RandomEffectDataset(type={self.config.random_effect_type}, shard={self.config.feature_shard_id},"
                f" entities={self.n_entities}, active rows={len(self.active_rows)}, passive rows="
                f"{len(self.passive_rows)}, buckets={len(self.buckets)}, mean projected dim="
                f"{float(d.mean()) if len(d) else 0:.1f})")
