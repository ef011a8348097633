"""Random-effect feature projectors.

Reference: ``photon-api/.../projector/{Projector,IndexMapProjector,IndexMapProjectorRDD,ProjectionMatrix,
IdentityProjector,ProjectorType}.scala``.

* ``INDEX_MAP``: per entity, compact the global feature ids that occur in its (active U passive) rows into a
  dense local index space (``IndexMapProjectorRDD.scala:166-207``). Represented for ALL entities at once as one
  entity-major sorted key array ``key = entity * D + feature`` (a CSR over entities), which is also what the
  vectorised scoring path (K6) searches.
* ``RANDOM(k)``: one Gaussian matrix shared by all entities, entries N(0,1)/k clipped to [-1, 1], plus an
  intercept row mapping the last original column (``ProjectionMatrix.scala:95-124``).
* ``IDENTITY``: the full shard dimension.
"""
from __future__ import annotations

import enum
from dataclasses import dataclass
from typing import Optional

import numpy as np

from ..constants import RANDOM_SEED


class ProjectorKind(str, enum.Enum):
    INDEX_MAP = "INDEX_MAP"
    RANDOM = "RANDOM"
    IDENTITY = "IDENTITY"


@dataclass(frozen=True)
class ProjectorType:
    kind: ProjectorKind = ProjectorKind.INDEX_MAP
    projected_dim: Optional[int] = None  # RANDOM only

    @staticmethod
    def parse(s) -> "ProjectorType":
        if isinstance(s, ProjectorType):
            return s
        s = str(s).strip().upper()
        if s.startswith("RANDOM"):
            k = int(s.split("=")[1]) if "=" in s else int(s[s.index("(") + 1:s.index(")")])
            return ProjectorType(ProjectorKind.RANDOM, k)
        return ProjectorType(ProjectorKind[s])

    def __str__(self):
        return f"RANDOM={self.projected_dim}" if self.kind == ProjectorKind.RANDOM else self.kind.value


INDEX_MAP = ProjectorType(ProjectorKind.INDEX_MAP)
IDENTITY = ProjectorType(ProjectorKind.IDENTITY)


def RandomProjection(k: int) -> ProjectorType:  # noqa: N802 (reference name)
    return ProjectorType(ProjectorKind.RANDOM, k)


class IndexMapProjection:
    """Entity-major compaction of active feature ids: ``ptr[E+1]``, ``feat[sum d_e]`` (sorted per entity).

    Built on the host (:meth:`build`) or from device-resident sorted keys (:meth:`from_sorted_keys`, the
    GPU dataset build); in the latter case ``keys`` / ``feat`` are copied to the host only when asked for."""

    def __init__(self, ptr: np.ndarray, feat: Optional[np.ndarray], dim: int, keys_t=None):
        self.ptr = ptr.astype(np.int64)
        self.dim = int(dim)
        self._keys_t = keys_t
        self._feat = None if feat is None else feat.astype(np.int64)
        self._keys = None
        if feat is not None:
            n_ent = len(ptr) - 1
            ent = np.repeat(np.arange(n_ent, dtype=np.int64), np.diff(self.ptr))
            self._keys = ent * self.dim + self._feat  # sorted ascending

    @staticmethod
    def from_sorted_keys(keys_t, n_entities: int, dim: int) -> "IndexMapProjection":
        import torch
        from ..ops.native import sorted_counts
        cnt = sorted_counts(keys_t // dim, n_entities)     # sorted keys: per-entity runs by binary search
        ptr = np.zeros(n_entities + 1, dtype=np.int64)
        ptr[1:] = np.cumsum(cnt.cpu().numpy())
        return IndexMapProjection(ptr, None, dim, keys_t=keys_t)

    @property
    def keys(self) -> np.ndarray:
        if self._keys is None:
            self._keys = self._keys_t.cpu().numpy()
        return self._keys

    @property
    def feat(self) -> np.ndarray:
        if self._feat is None:
            self._feat = self.keys % self.dim
        return self._feat

    @staticmethod
    def build(entity_of_entry: np.ndarray, feature_of_entry: np.ndarray, n_entities: int, dim: int):
        keys = np.unique(entity_of_entry.astype(np.int64) * dim + feature_of_entry.astype(np.int64))
        ent = keys // dim
        feat = keys % dim
        ptr = np.zeros(n_entities + 1, dtype=np.int64)
        np.add.at(ptr, ent + 1, 1)
        return IndexMapProjection(np.cumsum(ptr), feat, dim)

    def local_dims(self) -> np.ndarray:
        return np.diff(self.ptr)

    def local_index(self, entity: np.ndarray, feature: np.ndarray) -> np.ndarray:
        """Local index of (entity, feature) pairs; -1 when the feature is not in the entity's map."""
        k = entity.astype(np.int64) * self.dim + feature.astype(np.int64)
        pos = np.searchsorted(self.keys, k)
        pos_c = np.minimum(pos, len(self.keys) - 1) if len(self.keys) else pos
        ok = (pos < len(self.keys)) & (self.keys[pos_c] == k) if len(self.keys) else np.zeros(len(k), bool)
        return np.where(ok, pos - self.ptr[entity], -1)


def gaussian_projection_matrix(k: int, dim: int, keep_intercept: bool = True, seed: int = RANDOM_SEED):
    """``ProjectionMatrix.buildGaussianRandomProjectionMatrix``: [k(+1), dim]."""
    rng = np.random.default_rng(seed)
    m = rng.normal(size=(k, dim)) / k
    m = np.clip(m, -1.0, 1.0)
    if keep_intercept:
        row = np.zeros((1, dim))
        row[0, dim - 1] = 1.0
        m = np.vstack([m, row])
    return m
