"""Vector-space reductions used by the optimizers (dot, norm, any-non-zero, L1 norm, Gram matrix).

Every reduction an optimizer performs on a coefficient-sized vector goes through the ACTIVE space:

* :class:`LocalSpace` (default) — the vectors are whole; plain device reductions.
* :class:`ShardedSpace` — the vectors are FEATURE SHARDS (each rank holds a contiguous slice of w, g and the
  L-BFGS history, see :mod:`photon_ml_amd.parallel.feature_sharding`); each reduction is a local partial
  followed by one scalar all-reduce over the process group, and :meth:`gram` batches all the inner products of
  a set of vectors into ONE all-reduce (used by the vector-free L-BFGS two-loop in ``lbfgs.py``).

The space is selected with ``with active_space(space): ...`` around an optimizer run, so the optimizers
(L-BFGS, OWL-QN, TRON, line searches) are written once for both the replicated and the feature-sharded layouts.
The reference has no feature sharding (coefficients are broadcast whole: ``DistributedObjectiveFunction.scala:
57-58``, SURVEY §2.10 "Feature (column) sharding").
"""
from __future__ import annotations

import contextlib
import threading
from typing import Iterator, Sequence

import torch


class LocalSpace:
    sharded = False

    def dot(self, a: torch.Tensor, b: torch.Tensor) -> float:
        return float(torch.dot(a, b))

    def norm(self, a: torch.Tensor) -> float:
        return float(torch.linalg.vector_norm(a))

    def any_nonzero(self, a: torch.Tensor) -> bool:
        return bool(torch.any(a != 0))

    def all_zero(self, a: torch.Tensor) -> bool:
        return bool(torch.all(a == 0))

    def abs_sum(self, a: torch.Tensor) -> float:
        return float(torch.sum(torch.abs(a)))

    def dots(self, pairs) -> list:
        """Several inner products with ONE host synchronisation."""
        return torch.stack([torch.dot(a, b) for a, b in pairs]).to(torch.float64).tolist()

    def gram(self, vs: Sequence[torch.Tensor]) -> torch.Tensor:
        """Host fp64 matrix of all inner products ``vs[i] . vs[j]``."""
        return _gram_local(vs).to("cpu", torch.float64)


class ShardedSpace(LocalSpace):
    """Reductions over feature shards: local partial + all-reduce(sum / max) on ``group``."""

    sharded = True

    def __init__(self, group=None):
        self.group = group

    def _sum(self, t: torch.Tensor) -> torch.Tensor:
        import torch.distributed as dist
        from ..parallel.dist import is_dist
        if is_dist():
            dev = t.device if dist.get_backend(self.group) == "nccl" else torch.device("cpu")
            u = t.to(dev)
            dist.all_reduce(u, group=self.group)
            return u.to("cpu")
        return t.to("cpu")

    def dot(self, a, b) -> float:
        return float(self._sum(torch.dot(a, b).reshape(1).to(torch.float64))[0])

    def norm(self, a) -> float:
        return float(self._sum(torch.dot(a, a).reshape(1).to(torch.float64))[0]) ** 0.5

    def any_nonzero(self, a) -> bool:
        return float(self._sum(torch.any(a != 0).to(torch.float64).reshape(1))[0]) > 0

    def all_zero(self, a) -> bool:
        return not self.any_nonzero(a)

    def abs_sum(self, a) -> float:
        return float(self._sum(torch.sum(torch.abs(a)).reshape(1).to(torch.float64))[0])

    def dots(self, pairs) -> list:
        return self._sum(torch.stack([torch.dot(a, b) for a, b in pairs]).to(torch.float64)).tolist()

    def gram(self, vs):
        return self._sum(_gram_local(vs).to(torch.float64))


_GRAM_BLOCK = 1 << 14


def _gram_local(vs: Sequence[torch.Tensor]) -> torch.Tensor:
    """V V^T for a few (k ~ 21) very long vectors. A plain GEMM with K = D ~ 1e6-1e8 and a 21 x 21 output gives the
    BLAS one tile and no split-K (measured on MI355X: 160 ms per call at D = 1M, 281 ms at 10M); cut K into 16K blocks and
    batch them (one bmm of D / 16K independent 21 x 16K x 21 products; 2.8-2.9 ms at both sizes), then sum."""
    if vs and vs[0].is_cuda:
        from ..ops.native import gram
        G = gram(list(vs))          # one-pass LDS-tiled HIP kernel (ops/csrc/glm_kernels.hip gram_kernel)
        if G is not None:
            return G
    V = torch.stack(list(vs))
    k, n = V.shape
    if n <= 4 * _GRAM_BLOCK:
        return V @ V.T
    nb = -(-n // _GRAM_BLOCK)
    if nb * _GRAM_BLOCK != n:
        V = torch.nn.functional.pad(V, (0, nb * _GRAM_BLOCK - n))
    Vb = V.view(k, nb, _GRAM_BLOCK).transpose(0, 1)            # [nb, k, B]
    return torch.bmm(Vb, Vb.transpose(1, 2)).sum(0)


_LOCAL = LocalSpace()
_state = threading.local()


def current() -> LocalSpace:
    return getattr(_state, "space", None) or _LOCAL


@contextlib.contextmanager
def active_space(space: LocalSpace) -> Iterator[LocalSpace]:
    prev = getattr(_state, "space", None)
    _state.space = space
    try:
        yield space
    finally:
        _state.space = prev


def vdot(a, b) -> float:
    return current().dot(a, b)


def vdots(pairs) -> list:
    return current().dots(pairs)


def vnorm(a) -> float:
    return current().norm(a)
