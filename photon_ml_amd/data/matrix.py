"""Host-side sparse feature matrices (CSR) and labeled-data containers.

The reference keeps one Breeze ``SparseVector`` per ``LabeledPoint`` inside an RDD
(``photon-lib/.../data/LabeledPoint.scala:32-63``). Here a whole feature shard is ONE CSR matrix: rows are
samples, columns are feature indices of the shard's index map. Device residency (HBM) and the blocked layouts
used by the HIP kernels are built from this in ``photon_ml_amd/ops/sparse_layout.py``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np
import scipy.sparse as sp


class DeviceCSR:
    """A CSR feature shard resident on a device (torch tensors): what entity-sharded routing produces, handed to
    the device random-effect build and the scoring kernels without a host round trip. Minimal
    scipy-like surface (``shape``, ``nnz``, ``tocsr``, row subsets); :meth:`to_scipy` copies to the host for the
    host-only code paths."""

    def __init__(self, indptr, indices, data, shape, has_sorted_indices: bool = False):
        import torch
        self.indptr = indptr.to(torch.int64)
        self.indices = indices
        self.data = data.to(torch.float64)
        self.shape = (int(shape[0]), int(shape[1]))
        self.has_sorted_indices = bool(has_sorted_indices)
        self._pml_dev_cache = {}

    @property
    def device(self):
        return self.data.device

    @property
    def nnz(self) -> int:
        return int(self.data.numel())

    def tocsr(self):
        return self

    def offload_to_host(self) -> None:
        """Move the arrays to host memory in place (same object, CPU tensors): for a shard whose device layout has
        been built elsewhere (the fixed effect's tiled DeviceGLMData), so the routed copy does not double its HBM
        footprint for the rest of the fit. Later device consumers ``.to(device)`` it again."""
        self.indptr, self.indices, self.data = self.indptr.cpu(), self.indices.cpu(), self.data.cpu()
        self._pml_dev_cache = {}

    def to_scipy(self) -> sp.csr_matrix:
        m = sp.csr_matrix((self.data.cpu().numpy(), self.indices.cpu().numpy().astype(np.int32, copy=False),
                           self.indptr.cpu().numpy()), shape=self.shape)
        m.has_sorted_indices = self.has_sorted_indices
        return m

    def __getitem__(self, rows) -> "DeviceCSR":
        """Row subset (an index array / mask over rows), gathered on the device."""
        import torch
        dev = self.data.device
        r = torch.as_tensor(np.asarray(rows) if not isinstance(rows, torch.Tensor) else rows, device=dev)
        if r.dtype == torch.bool:
            r = torch.nonzero(r).squeeze(1)
        r = r.to(torch.int64)
        lens = (self.indptr[1:] - self.indptr[:-1])[r]
        ip = torch.zeros(r.numel() + 1, dtype=torch.int64, device=dev)
        torch.cumsum(lens, 0, out=ip[1:])
        tot = int(ip[-1])
        src = torch.repeat_interleave(self.indptr[:-1][r] - ip[:-1], lens, output_size=tot)
        src += torch.arange(tot, device=dev)
        return DeviceCSR(ip, self.indices[src], self.data[src], (r.numel(), self.shape[1]), self.has_sorted_indices)


def as_csr(x, n_cols: Optional[int] = None) -> sp.csr_matrix:
    """Coerce dense arrays / scipy matrices to canonical float64 CSR with sorted indices (device-resident
    :class:`DeviceCSR` shards pass through unchanged)."""
    if isinstance(x, DeviceCSR):
        return x
    if sp.issparse(x):
        m = x.tocsr().astype(np.float64, copy=False)     # no copy of an fp64 CSR (8 GB+ at GAME config 5)
    else:
        m = sp.csr_matrix(np.asarray(x, dtype=np.float64))
    if n_cols is not None and m.shape[1] != n_cols:
        m = sp.csr_matrix((m.data, m.indices, m.indptr), shape=(m.shape[0], n_cols))
    m.sum_duplicates()
    m.sort_indices()
    return m


def csr_from_rows(rows: Sequence[tuple], n_cols: int) -> sp.csr_matrix:
    """Build CSR from ``[(indices, values), ...]``."""
    indptr = np.zeros(len(rows) + 1, dtype=np.int64)
    for i, (idx, _) in enumerate(rows):
        indptr[i + 1] = indptr[i] + len(idx)
    indices = np.empty(indptr[-1], dtype=np.int32)
    values = np.empty(indptr[-1], dtype=np.float64)
    for i, (idx, val) in enumerate(rows):
        indices[indptr[i]:indptr[i + 1]] = idx
        values[indptr[i]:indptr[i + 1]] = val
    return as_csr(sp.csr_matrix((values, indices, indptr), shape=(len(rows), n_cols)))


@dataclass
class LabeledData:
    """A batch of labeled samples for ONE feature shard (the GLM view).

    ``x`` is CSR [N, D]; ``y``/``offsets``/``weights`` are float64 [N]; ``uids`` int64 [N] (unique sample ids,
    ``GameConverters.scala:53-59`` assigns them by ``zipWithIndex``).
    """

    x: sp.csr_matrix
    y: np.ndarray
    offsets: Optional[np.ndarray] = None
    weights: Optional[np.ndarray] = None
    uids: Optional[np.ndarray] = None

    def __post_init__(self):
        self.x = as_csr(self.x)
        n = self.x.shape[0]
        self.y = np.asarray(self.y, dtype=np.float64).reshape(n)
        self.offsets = np.zeros(n) if self.offsets is None else np.asarray(self.offsets, np.float64).reshape(n)
        self.weights = np.ones(n) if self.weights is None else np.asarray(self.weights, np.float64).reshape(n)
        self.uids = np.arange(n, dtype=np.int64) if self.uids is None else np.asarray(self.uids, np.int64)

    @property
    def n_rows(self) -> int:
        return self.x.shape[0]

    @property
    def n_features(self) -> int:
        return self.x.shape[1]

    def subset(self, rows) -> "LabeledData":
        rows = np.asarray(rows)
        return LabeledData(self.x[rows], self.y[rows], self.offsets[rows], self.weights[rows], self.uids[rows])

    def with_offsets(self, offsets: np.ndarray) -> "LabeledData":
        return LabeledData(self.x, self.y, offsets, self.weights, self.uids)

    def with_weights(self, weights: np.ndarray) -> "LabeledData":
        return LabeledData(self.x, self.y, self.offsets, weights, self.uids)
