"""Per-feature statistics (``photon-lib/.../stat/BasicStatisticalSummary.scala:36-117``, MLlib colStats semantics).

mean, unbiased variance, count, numNonzeros, max, min (implicit zeros included when a column is not dense), L1 and
L2 norms and mean |x|; invalid (NaN / Inf / negative) variances are reset to 1.0 with a warning. Computed with
sparse column reductions (K9); with a process group the sufficient statistics are all-reduced (C24).
"""
from __future__ import annotations

import logging
from dataclasses import dataclass

import numpy as np
import scipy.sparse as sp
import torch

log = logging.getLogger(__name__)


@dataclass
class BasicStatisticalSummary:
    mean: torch.Tensor
    variance: torch.Tensor
    count: int
    num_nonzeros: torch.Tensor
    max: torch.Tensor
    min: torch.Tensor
    norm_l1: torch.Tensor
    norm_l2: torch.Tensor
    mean_abs: torch.Tensor

    @staticmethod
    def from_sufficient(count, s1, s2, sabs, nnz, mx, mn) -> "BasicStatisticalSummary":
        n = float(count)
        mean = s1 / n if n > 0 else s1
        var = (s2 - n * mean * mean) / (n - 1) if n > 1 else np.zeros_like(s1)
        # implicit zeros participate in max/min when a column has fewer non-zeros than rows
        mx = np.where(nnz < n, np.maximum(mx, 0.0), mx)
        mn = np.where(nnz < n, np.minimum(mn, 0.0), mn)
        bad = ~np.isfinite(var) | (var < 0)
        if bad.any():
            log.warning("Found %d features where variance was either non-positive, not-a-number, or infinite. "
                        "The variances for these features have been re-set to 1.0.", int(bad.sum()))
            var = np.where(bad, 1.0, var)
        t = lambda a: torch.from_numpy(np.asarray(a, dtype=np.float64))
        return BasicStatisticalSummary(t(mean), t(var), int(count), t(nnz), t(mx), t(mn), t(sabs), t(np.sqrt(s2)),
                                       t(sabs / n if n > 0 else sabs))

    @staticmethod
    def compute(x: sp.csr_matrix, all_reduce: bool = False) -> "BasicStatisticalSummary":
        x = x.tocsc()
        n, d = x.shape
        s1 = np.asarray(x.sum(axis=0)).ravel()
        s2 = np.asarray(x.multiply(x).sum(axis=0)).ravel()
        sabs = np.asarray(abs(x).sum(axis=0)).ravel()
        nnz = np.diff(x.indptr).astype(np.float64)
        mx = np.full(d, -np.inf)
        mn = np.full(d, np.inf)
        if x.nnz:
            col = np.repeat(np.arange(d), np.diff(x.indptr))
            np.maximum.at(mx, col, x.data)
            np.minimum.at(mn, col, x.data)
        mx = np.where(np.isinf(mx), 0.0, mx)
        mn = np.where(np.isinf(mn), 0.0, mn)
        count = n
        if all_reduce:
            from ..parallel.dist import is_dist
            import torch.distributed as dist
            if is_dist():
                buf = torch.from_numpy(np.concatenate([[count], s1, s2, sabs, nnz]).astype(np.float64))
                dist.all_reduce(buf)
                b = buf.numpy()
                count, s1, s2, sabs, nnz = int(b[0]), b[1:1 + d], b[1 + d:1 + 2 * d], b[1 + 2 * d:1 + 3 * d], b[1 + 3 * d:]
                tmx, tmn = torch.from_numpy(mx), torch.from_numpy(mn)
                dist.all_reduce(tmx, op=dist.ReduceOp.MAX)
                dist.all_reduce(tmn, op=dist.ReduceOp.MIN)
                mx, mn = tmx.numpy(), tmn.numpy()
        return BasicStatisticalSummary.from_sufficient(count, s1, s2, sabs, nnz, mx, mn)

    @staticmethod
    def from_device(data, all_reduce: bool = False) -> "BasicStatisticalSummary":
        """Same statistics straight from a device-resident shard (``ops.device.DeviceGLMData``, tiled layout):
        column reductions over the forward streams with device scatter-reductions, no host copy of the
        non-zeros (K9 on the GPU); with ``all_reduce`` the sufficient statistics are reduced over the process
        group (C24). Feature order: original (the device relabelling is undone)."""
        dev = data.device
        d = data.dim
        f64 = torch.float64
        s1 = torch.zeros(d, dtype=f64, device=dev)
        s2 = torch.zeros(d, dtype=f64, device=dev)
        sabs = torch.zeros(d, dtype=f64, device=dev)
        nnz = torch.zeros(d, dtype=f64, device=dev)
        mx = torch.full((d,), float("-inf"), dtype=f64, device=dev)
        mn = torch.full((d,), float("inf"), dtype=f64, device=dev)
        for c, ch in enumerate(data.csr):
            if getattr(ch, "kind", None) != "tl":
                raise ValueError("from_device needs the tiled layout")
            pk, vl = ch.logical()
            col = (pk.to(torch.int64) >> ch.rbits) + data.col_lo[c]     # logical(): non-negative int64
            v = vl.to(f64)
            s1.index_add_(0, col, v)
            s2.index_add_(0, col, v * v)
            sabs.index_add_(0, col, v.abs())
            nnz.index_add_(0, col, torch.ones_like(v))
            mx.scatter_reduce_(0, col, v, "amax")
            mn.scatter_reduce_(0, col, v, "amin")
            del pk, vl, col, v
        if data.old_of_new is not None:   # device column j is original feature old_of_new[j]
            def unperm(t):
                out = torch.empty_like(t)
                out[data.old_of_new] = t
                return out
            s1, s2, sabs, nnz, mx, mn = (unperm(t) for t in (s1, s2, sabs, nnz, mx, mn))
        count = float(data.n_rows)
        if all_reduce:
            from ..parallel.dist import is_dist
            import torch.distributed as dist
            if is_dist():
                cdev = dev if dist.get_backend() == "nccl" else torch.device("cpu")
                buf = torch.cat([torch.tensor([count], dtype=f64, device=dev), s1, s2, sabs, nnz]).to(cdev)
                dist.all_reduce(buf)
                count = float(buf[0])
                s1, s2, sabs, nnz = (t.to(dev) for t in buf[1:].split(d))
                tmx, tmn = mx.to(cdev), mn.to(cdev)
                dist.all_reduce(tmx, op=dist.ReduceOp.MAX)
                dist.all_reduce(tmn, op=dist.ReduceOp.MIN)
                mx, mn = tmx.to(dev), tmn.to(dev)
        mx = torch.where(torch.isinf(mx), torch.zeros_like(mx), mx)
        mn = torch.where(torch.isinf(mn), torch.zeros_like(mn), mn)
        h = lambda t: t.cpu().numpy()
        return BasicStatisticalSummary.from_sufficient(int(count), h(s1), h(s2), h(sabs), h(nnz), h(mx), h(mn))

