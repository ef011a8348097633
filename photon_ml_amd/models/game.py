"""GAME models: fixed-effect model, random-effect model, GameModel.

Reference: ``photon-api/.../model/FixedEffectModel.scala:31-145`` (broadcast GLM + shard id, scoring = dot
product), ``RandomEffectModel.scala:38-298`` (RDD of per-entity GLMs; scoring is a partitioned hash join),
``photon-lib/.../model/GameModel.scala:32-170`` (coordinate -> model map, a single task type enforced) and
``DatumScoringModel.scala``.

Random-effect models are stored entity-major in the ORIGINAL feature space as one sorted key array
``key = entity_index * D + feature`` with values (and optional variances) — a CSR over entities. On the GPU,
scoring (K5 fixed effect, K6 random effect) is the ``score_rows_kernel`` HIP kernel (``ops/csrc/game_kernels.hip``:
16 lanes per sample row, per-lane binary search in the row's entity segment, fixed-order reduction); on the host
it is one vectorised ``searchsorted`` of the sample non-zeros' keys. No per-entity Python objects, no joins.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, Iterable, Optional

import numpy as np
import scipy.sparse as sp
import torch

from ..constants import TaskType
from ..data.matrix import DeviceCSR
from .glm import Coefficients, GeneralizedLinearModel, model_for_task


def _csr_to_torch(x: sp.csr_matrix, device):
    """(row, col, val, indptr) device tensors of a CSR shard, cached ON the matrix object per device: validation
    data is scored after every coordinate update (``CoordinateDescent._score_validation``), and re-uploading
    24 B/nnz each time would dominate scoring a large validation set."""
    dev = torch.device(device)
    cache = getattr(x, "_pml_dev_cache", None)
    if cache is None:
        cache = {}
        try:
            x._pml_dev_cache = cache
        except AttributeError:  # pragma: no cover - exotic sparse subclasses
            pass
    key = str(dev)
    if key not in cache and isinstance(x, DeviceCSR):
        ip = x.indptr.to(dev)
        row = torch.repeat_interleave(torch.arange(x.shape[0], device=dev), ip[1:] - ip[:-1], output_size=x.nnz)
        cache[key] = (row, x.indices.to(dev, torch.int64), x.data.to(dev), ip)
    if key not in cache:
        x = x.tocsr()
        indptr = np.asarray(x.indptr, dtype=np.int64)
        row = np.repeat(np.arange(x.shape[0], dtype=np.int64), np.diff(indptr))
        cache[key] = (torch.from_numpy(row).to(dev), torch.from_numpy(x.indices.astype(np.int64)).to(dev),
                      torch.from_numpy(x.data.astype(np.float64)).to(dev), torch.from_numpy(indptr).to(dev))
    return cache[key]


def _csr_col32(x: sp.csr_matrix, device) -> torch.Tensor:
    """int32 column ids of a cached device CSR (the scoring kernel's index type), cached beside it."""
    dev = torch.device(device)
    col = _csr_to_torch(x, dev)[1]
    cache = getattr(x, "_pml_dev_cache", None)
    key = "col32:" + str(dev)
    if cache is None:
        return col.to(torch.int32)
    if key not in cache:
        cache[key] = col.to(torch.int32)
    return cache[key]


def _use_kernel(dev: torch.device) -> bool:
    return dev.type == "cuda"


def _row_sums(contrib: torch.Tensor, row: torch.Tensor, indptr: torch.Tensor, n: int) -> torch.Tensor:
    """Per-row sums of CSR-ordered per-entry values, fp64. On the GPU a segmented reduction over the CSR row
    pointer (deterministic: no atomics, unlike ``index_add_``)."""
    if contrib.is_cuda and contrib.numel() > 0:
        return torch.segment_reduce(contrib, "sum", offsets=indptr, unsafe=True)
    return torch.zeros(n, dtype=torch.float64, device=contrib.device).index_add_(0, row, contrib)


class FixedEffectModel:
    def __init__(self, glm: GeneralizedLinearModel, feature_shard_id: str):
        self.glm = glm
        self.feature_shard_id = feature_shard_id

    @property
    def task(self) -> TaskType:
        return self.glm.task

    def score(self, data, device="cpu") -> torch.Tensor:
        x = data.shard(self.feature_shard_id)
        means = self.glm.coefficients.means
        if x.shape[1] != means.numel():
            raise ValueError(f"shard {self.feature_shard_id} dim {x.shape[1]} != model dim {means.numel()}")
        dev = torch.device(device)
        if dev.type == "cpu" and not isinstance(x, DeviceCSR):
            w = means.cpu().numpy()
            return torch.from_numpy(np.asarray(x @ w).reshape(-1))
        row, col, val, indptr = _csr_to_torch(x, dev)
        if _use_kernel(dev):
            from ..ops.native import score_rows
            return score_rows(indptr, _csr_col32(x, dev), val, means.to(dev, torch.float64).contiguous())
        return _row_sums(val * means.to(dev, torch.float64)[col], row, indptr, x.shape[0])

    def __repr__(self):
        return f"FixedEffectModel(shard={self.feature_shard_id}, dim={self.glm.coefficients.dim})"


class RandomEffectModel:
    """Per-entity GLMs of one random-effect coordinate, stored entity-major as sorted ``key = entity * dim +
    feature`` with values (and optional variances) — the whole coordinate's models as three flat arrays.

    The arrays may be numpy (host) or torch tensors (e.g. device-resident, straight out of the block-diagonal
    solver): ``keys`` / ``values`` / ``variances`` give host numpy views (copied from the device once, lazily),
    ``tensors(device)`` gives torch tensors without a host round trip (scoring, regularization term, warm start).
    """

    def __init__(self, random_effect_type: str, feature_shard_id: str, task: TaskType, entity_ids: np.ndarray,
                 dim: int, keys, values, variances=None, sum_sq: Optional[float] = None):
        """``values`` may be a zero-argument callable producing the device values on first use (with device
        ``keys``): the row-space random-effect solve returns its primal coefficients lazily, because inside
        coordinate descent only the scores (L beta) and ||w||^2 = ||beta||^2 (``sum_sq``) are needed — the
        transpose pass that builds w runs only when the model itself is read (validation scoring, save, warm
        start of another coordinate)."""
        self.random_effect_type = random_effect_type
        self.feature_shard_id = feature_shard_id
        self._task = TaskType.parse(task)
        self.entity_ids = np.asarray(entity_ids)
        self.dim = int(dim)
        self._host = None
        self._dev = None
        self._lazy = None
        self._sum_sq = sum_sq
        if isinstance(keys, torch.Tensor):
            # solver output: keys already sorted (entity-major projection order)
            if callable(values):
                self._lazy = values
                values = None
            self._dev = (keys.to(torch.int64), None if values is None else values.to(torch.float64),
                         None if variances is None else variances.to(torch.float64))
            return
        keys = np.asarray(keys, dtype=np.int64)
        values = np.asarray(values, dtype=np.float64)
        if len(keys) > 1 and not bool(np.all(keys[1:] >= keys[:-1])):  # solvers emit sorted keys: skip the sort
            order = np.argsort(keys, kind="stable")
            keys, values = keys[order], values[order]
            if variances is not None:
                variances = np.asarray(variances)[order]
        self._host = (keys, values, None if variances is None else np.asarray(variances, dtype=np.float64))

    def _d(self):
        if self._lazy is not None:
            k, _, var = self._dev
            self._dev = (k, self._lazy().to(torch.float64), var)
            self._lazy = None
        return self._dev

    def materialize(self) -> "RandomEffectModel":
        """Produce lazily deferred coefficients now (on the device)."""
        self._d()
        return self

    @property
    def materialized(self) -> bool:
        return self._lazy is None

    def _h(self):
        if self._host is None:
            k, v, var = self._d()
            self._host = (k.cpu().numpy(), v.cpu().numpy(), None if var is None else var.cpu().numpy())
        return self._host

    @property
    def keys(self) -> np.ndarray:
        return self._h()[0]

    @property
    def values(self) -> np.ndarray:
        return self._h()[1]

    @property
    def variances(self) -> Optional[np.ndarray]:
        if self._host is None and self._dev is not None and self._dev[2] is None:
            return None
        return self._h()[2]

    @property
    def nnz(self) -> int:
        return int(self._dev[0].numel()) if self._dev is not None else len(self._host[0])

    def tensors(self, device):
        """(keys, values) as torch tensors on ``device`` (no host copy when already resident there)."""
        dev = torch.device(device)
        if self._dev is not None:
            k, v, _ = self._d()
            return k.to(dev), v.to(dev)
        return torch.from_numpy(self._host[0]).to(dev), torch.from_numpy(self._host[1]).to(dev)

    def sum_abs_and_sq(self, need_abs: bool = True):
        """(sum |w|, sum w^2) over all coefficients (regularization term value), computed where they live.
        ``need_abs=False`` on a lazy model returns (nan, ||beta||^2) without materialising it."""
        if self._lazy is not None and not need_abs and self._sum_sq is not None:
            return float("nan"), float(self._sum_sq)
        if self._dev is not None:
            v = self._d()[1]   # reductions without model-sized temporaries (1.25e9 coefficients at config 5)
            return float(torch.linalg.vector_norm(v, 1)), float(torch.linalg.vector_norm(v, 2)) ** 2
        v = self._host[1]
        return float(np.abs(v).sum()), float((v * v).sum())

    @property
    def task(self) -> TaskType:
        return self._task

    @property
    def n_entities(self) -> int:
        return len(self.entity_ids)

    def entity_index(self, ids: np.ndarray) -> np.ndarray:
        ids = np.asarray(ids)
        ids_s = ids.astype(str) if ids.dtype == object else ids
        ent = self.entity_ids
        pos = np.searchsorted(ent, ids_s)
        pos_c = np.minimum(pos, max(len(ent) - 1, 0))
        ok = (pos < len(ent)) & (ent[pos_c] == ids_s) if len(ent) else np.zeros(len(ids_s), bool)
        return np.where(ok, pos, -1)

    def coefficients_of(self, entity_id) -> Coefficients:
        e = int(self.entity_index(np.array([entity_id]))[0])
        if e < 0:
            raise KeyError(entity_id)
        lo, hi = np.searchsorted(self.keys, [e * self.dim, (e + 1) * self.dim])
        means = np.zeros(self.dim)
        means[self.keys[lo:hi] - e * self.dim] = self.values[lo:hi]
        var = None
        if self.variances is not None:
            var = np.zeros(self.dim)
            var[self.keys[lo:hi] - e * self.dim] = self.variances[lo:hi]
        return Coefficients(torch.from_numpy(means), None if var is None else torch.from_numpy(var))

    def models(self) -> Iterable:
        """Yield (entity_id, GLM) pairs (for IO / inspection)."""
        for i, eid in enumerate(self.entity_ids):
            yield eid, model_for_task(self._task, self.coefficients_of(eid))

    def entity_csr(self, device):
        """Entity-major CSR of the model on ``device``: (eptr [E + 1] int64, sorted feature ids int32, values f64),
        cached per device (models are immutable once built)."""
        dev = torch.device(device)
        cache = self.__dict__.setdefault("_ecsr", {})
        if str(dev) not in cache:
            keys, vals = self.tensors(dev)
            ent = torch.div(keys, self.dim, rounding_mode="floor")
            bounds = torch.arange(self.n_entities + 1, device=dev, dtype=torch.int64) * self.dim
            eptr = torch.searchsorted(keys, bounds)
            cache[str(dev)] = (eptr, (keys - ent * self.dim).to(torch.int32), vals.contiguous())
        return cache[str(dev)]

    def _row_entities(self, data, dev) -> torch.Tensor:
        """Model entity index of every sample row (-1: no model), int32 on ``dev``; cached on the data object for
        this entity table (validation data is scored after every coordinate update)."""
        cache = data.__dict__.setdefault("_pml_ent_cache", {})
        ids = self.entity_ids
        key = (self.random_effect_type, id(ids), len(ids), str(dev))
        hit = cache.get(key)
        if hit is None or hit[0] is not ids:
            ent = self.entity_index(data.id_tags[self.random_effect_type]).astype(np.int32)
            hit = (ids, torch.from_numpy(ent).to(dev))
            cache[key] = hit
        return hit[1]

    def score(self, data, device="cpu", mask: Optional[np.ndarray] = None) -> torch.Tensor:
        """Score every sample whose entity has a model (K6): sum_j x_ij * w_{e(i), j}."""
        x = data.shard(self.feature_shard_id)
        n = x.shape[0]
        if self.nnz == 0:
            return torch.zeros(n, dtype=torch.float64, device=device)
        dev = torch.device(device)
        if _use_kernel(dev):
            from ..ops.native import score_rows
            row, col, val, indptr = _csr_to_torch(x, dev)
            ent_t = self._row_entities(data, dev)
            if mask is not None:
                ent_t = torch.where(torch.from_numpy(np.asarray(mask, dtype=bool)).to(dev), ent_t,
                                    torch.full_like(ent_t, -1))
            eptr, efeat, vals = self.entity_csr(dev)
            return score_rows(indptr, _csr_col32(x, dev), val, vals, ent_t.contiguous(), eptr, efeat)
        ent = self.entity_index(data.id_tags[self.random_effect_type])
        if mask is not None:
            ent = np.where(mask, ent, -1)
        row, col, val, indptr = _csr_to_torch(x, dev)
        ent_t = torch.from_numpy(ent).to(dev)
        e = ent_t[row]
        keys, vals = self.tensors(dev)
        out = torch.zeros(n, dtype=torch.float64, device=dev)
        if keys.numel() == 0 or row.numel() == 0:
            return out
        k = e * self.dim + col
        pos = torch.searchsorted(keys, k).clamp(max=keys.numel() - 1)
        hit = (keys[pos] == k) & (e >= 0)
        contrib = torch.where(hit, val * vals[pos], torch.zeros_like(val))
        if dev.type == "cpu":
            return out.index_add_(0, row, contrib)
        return _row_sums(contrib, row, indptr, n)

    def __repr__(self):
        return (f"RandomEffectModel(type={self.random_effect_type}, shard={self.feature_shard_id}, "
                f"entities={self.n_entities}, nnz={self.nnz})")


class GameModel:
    """Ordered map coordinate id -> model; all sub-models must share one task type."""

    def __init__(self, models: "OrderedDict[str, object]"):
        self.models = OrderedDict(models)
        tasks = {m.task for m in self.models.values()}
        if len(tasks) > 1:
            raise ValueError(f"GameModel sub-models have different task types: {tasks}")
        self.task = tasks.pop() if tasks else TaskType.NONE

    def get(self, coordinate_id: str):
        return self.models.get(coordinate_id)

    def updated(self, coordinate_id: str, model) -> "GameModel":
        m = OrderedDict(self.models)
        m[coordinate_id] = model
        return GameModel(m)

    def score(self, data, device="cpu") -> torch.Tensor:
        """Sum of every coordinate's scores (no offsets)."""
        total = torch.zeros(data.n_rows, dtype=torch.float64, device=device)
        for m in self.models.values():
            total = total + m.score(data, device)
        return total

    def __iter__(self):
        return iter(self.models.items())

    def __repr__(self):
        return "GameModel(" + ", ".join(f"{k}: {v}" for k, v in self.models.items()) + ")"
