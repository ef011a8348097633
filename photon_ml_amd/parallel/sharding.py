"""Entity sharding and residual routing for multi-GPU GAME (SURVEY §2.9 C8-C12, §2.10 entity parallelism).

Reference: ``photon-api/.../data/RandomEffectDataSetPartitioner.scala:42-148`` (count rows per entity, take the
10,000 largest, greedily bin-pack them onto the least-loaded partition with a min-heap, hash the rest),
``RandomEffectDataSet.scala:68-88, 239-315`` (groupByKey of rows by entity, ``addScoresToOffsets`` = join +
groupByKey every update) and ``RandomEffectCoordinate.scala:157-187`` (scores re-partitioned by uid).

MI355X design: rows stay in their sample shard for the fixed effects; for each random-effect coordinate every row
is ROUTED ONCE to the GPU that owns its entity (one variable-size all-to-all of the feature rows at build time,
C8). The permutation is kept, so each coordinate update moves only N-length fp64 vectors: partial scores to the
owners (C11) and new scores back (C12) — two ``all_to_all_single`` calls over xGMI per RE update instead of two
shuffles. Entity ownership is computed identically on every rank from all-gathered (entity key, count) pairs
(C9), so no broadcast is needed.
"""
from __future__ import annotations

import heapq
from typing import List, Optional, Sequence, Tuple

import numpy as np
import scipy.sparse as sp
import torch
import torch.distributed as dist

from .dist import is_dist, rank as _rank, world_size as _world

TOP_ENTITIES = 10_000


def stable_hash64(ids: np.ndarray) -> np.ndarray:
    """Deterministic 64-bit key of each entity id (same on every rank / run; pandas' SipHash with a fixed key)."""
    import pandas as pd
    ids = np.asarray(ids)
    if ids.dtype.kind in "iu":
        return pd.util.hash_array(ids.astype(np.int64)).view(np.int64)
    return pd.util.hash_array(ids.astype(str).astype(object)).view(np.int64)


def comm_device(group=None) -> torch.device:
    if is_dist() and dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def all_gather_varlen(t: torch.Tensor, group=None) -> List[torch.Tensor]:
    """All-gather 1-D tensors of different lengths (pads to the max length)."""
    if not is_dist():
        return [t]
    dev = comm_device(group)
    n = torch.tensor([t.numel()], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(_world())]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    m = max(sizes) if sizes else 0
    buf = torch.zeros(m, dtype=t.dtype, device=dev)
    buf[: t.numel()] = t.to(dev)
    outs = [torch.zeros_like(buf) for _ in range(_world())]
    dist.all_gather(outs, buf, group=group)
    return [o[:s].to(t.device) for o, s in zip(outs, sizes)]


def all_to_all_varlen(send: torch.Tensor, send_counts: Sequence[int], group=None) -> Tuple[torch.Tensor, List[int]]:
    """Variable-size all-to-all along dim 0 (rows already grouped by destination rank)."""
    if not is_dist():
        return send, list(send_counts)
    dev = comm_device(group)
    sc = torch.tensor(list(send_counts), dtype=torch.int64, device=dev)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc, group=group)
    recv_counts = [int(x) for x in rc.tolist()]
    tail = tuple(send.shape[1:])
    out = torch.empty((sum(recv_counts),) + tail, dtype=send.dtype, device=dev)
    dist.all_to_all_single(out, send.to(dev).contiguous(), recv_counts, list(send_counts), group=group)
    return out.to(send.device), recv_counts


class EntityPartitioner:
    """Entity key -> owning rank: greedy least-loaded bin packing of the largest entities, hash for the rest."""

    def __init__(self, keys: np.ndarray, counts: np.ndarray, n_parts: int, top_k: int = TOP_ENTITIES):
        self.n_parts = n_parts
        order = np.lexsort((keys, -counts))  # count desc, key asc: identical on every rank
        top = order[:top_k]
        heap = [(0, p) for p in range(n_parts)]
        heapq.heapify(heap)
        owner = {}
        for i in top:
            load, p = heapq.heappop(heap)
            owner[int(keys[i])] = p
            heapq.heappush(heap, (load + int(counts[i]), p))
        self.top_keys = np.fromiter(owner.keys(), dtype=np.int64, count=len(owner))
        self.top_owner = np.fromiter(owner.values(), dtype=np.int64, count=len(owner))
        srt = np.argsort(self.top_keys)
        self.top_keys, self.top_owner = self.top_keys[srt], self.top_owner[srt]

    def owner(self, keys: np.ndarray) -> np.ndarray:
        keys = np.asarray(keys, dtype=np.int64)
        out = (keys.view(np.uint64) % np.uint64(self.n_parts)).astype(np.int64)
        if len(self.top_keys):
            pos = np.searchsorted(self.top_keys, keys)
            pos_c = np.minimum(pos, len(self.top_keys) - 1)
            hit = self.top_keys[pos_c] == keys
            out[hit] = self.top_owner[pos_c[hit]]
        return out

    @staticmethod
    def build(local_keys: np.ndarray, group=None, top_k: int = TOP_ENTITIES) -> "EntityPartitioner":
        """All-gather per-rank (key, count) histograms (C9) and build the same partitioner everywhere."""
        uk, cnt = np.unique(np.asarray(local_keys, dtype=np.int64), return_counts=True)
        ks = all_gather_varlen(torch.from_numpy(uk), group)
        cs = all_gather_varlen(torch.from_numpy(cnt.astype(np.int64)), group)
        keys = torch.cat(ks).numpy()
        counts = torch.cat(cs).numpy()
        gk, inv = np.unique(keys, return_inverse=True)
        gc = np.bincount(inv, weights=counts).astype(np.int64)
        return EntityPartitioner(gk, gc, _world(), top_k)


class RowRouter:
    """Fixed permutation between this rank's sample rows and the rows it owns after routing by ``dest``.

    ``forward(v)``: local sample order -> concatenation over source ranks of the rows sent here (owner order);
    ``backward(u)``: the inverse (owner order -> local sample order). Both are one ``all_to_all_single``.

    Vectors stay where they are: the permutation is cached on each device it is used on, and under RCCL (``nccl``
    backend) the all-to-all runs directly on device tensors — an RE update moves its N-length score vectors
    GPU to GPU over xGMI with no host staging (C11/C12). Only the gloo backend (CPU rehearsals) stages through host
    memory, because gloo collectives take CPU tensors.
    """

    def __init__(self, dest: np.ndarray, group=None):
        self.group = group
        dest = np.asarray(dest, dtype=np.int64)
        self.n_local = len(dest)
        P = _world()
        self.perm = np.argsort(dest, kind="stable")          # local rows grouped by destination
        self.send_counts = np.bincount(dest, minlength=P).tolist()
        # exchange counts
        if is_dist():
            dev = comm_device(group)
            sc = torch.tensor(self.send_counts, dtype=torch.int64, device=dev)
            rc = torch.empty_like(sc)
            dist.all_to_all_single(rc, sc, group=group)
            self.recv_counts = [int(x) for x in rc.tolist()]
        else:
            self.recv_counts = list(self.send_counts)
        self.n_recv = int(sum(self.recv_counts))
        self.src_rank = np.repeat(np.arange(P), self.recv_counts)
        self._perm_on = {}

    def perm_on(self, device) -> torch.Tensor:
        """The routing permutation as an int64 tensor on ``device`` (uploaded once per device)."""
        key = str(torch.device(device))
        if key not in self._perm_on:
            self._perm_on[key] = torch.from_numpy(self.perm).to(device)
        return self._perm_on[key]

    def forward(self, v) -> torch.Tensor:
        t = torch.as_tensor(v)
        send = t[self.perm_on(t.device)]
        if not is_dist():
            return send
        out, _ = self._a2a(send, self.send_counts, self.recv_counts)
        return out

    def backward(self, u) -> torch.Tensor:
        t = torch.as_tensor(u)
        if is_dist():
            t, _ = self._a2a(t, self.recv_counts, self.send_counts)
        out = torch.empty_like(t)
        out[self.perm_on(t.device)] = t
        return out

    def _a2a(self, send: torch.Tensor, sc: List[int], rc: List[int]):
        dev = comm_device(self.group)
        tail = tuple(send.shape[1:])
        out = torch.empty((sum(rc),) + tail, dtype=send.dtype, device=dev)
        dist.all_to_all_single(out, send.to(dev).contiguous(), rc, sc, group=self.group)
        return out.to(send.device), rc

    def forward_csr(self, x: sp.csr_matrix) -> sp.csr_matrix:
        """Route sparse rows: one all-to-all each for row lengths, column indices and values. The entry
        permutation runs with torch ops on the communication device (the GPU under RCCL, so the gathers of the
        1G-entry shards of config 5 are device work and the collectives move device tensors)."""
        x = x.tocsr()
        dev = comm_device(self.group)
        indptr = torch.from_numpy(x.indptr.astype(np.int64)).to(dev)
        lens = indptr[1:] - indptr[:-1]
        perm = self.perm_on(dev)
        ol = lens[perm]
        tot = int(ol.sum())
        start = torch.cumsum(ol, 0) - ol
        ent = torch.repeat_interleave(indptr[:-1][perm] - start, ol, output_size=tot) + torch.arange(tot, device=dev)
        ri = torch.from_numpy(x.indices).to(dev)[ent].to(torch.int64)
        rv = torch.from_numpy(x.data).to(dev, torch.float64)[ent]
        del ent
        sc = torch.tensor(self.send_counts, dtype=torch.int64, device=dev)
        seg = torch.repeat_interleave(torch.arange(len(self.send_counts), device=dev), sc, output_size=perm.numel())
        nnz_send = torch.zeros(len(self.send_counts), dtype=torch.int64, device=dev).index_add_(0, seg, ol).tolist()
        rl = self.forward(lens)
        rseg = torch.repeat_interleave(torch.arange(len(self.recv_counts), device=dev),
                                       torch.tensor(self.recv_counts, dtype=torch.int64, device=dev),
                                       output_size=rl.numel())
        nnz_recv = torch.zeros(len(self.recv_counts), dtype=torch.int64, device=dev).index_add_(0, rseg, rl).tolist()
        if is_dist():
            ri, _ = self._a2a(ri, nnz_send, nnz_recv)
            rv, _ = self._a2a(rv, nnz_send, nnz_recv)
        rip = torch.zeros(rl.numel() + 1, dtype=torch.int64, device=dev)
        torch.cumsum(rl, 0, out=rip[1:])
        out = sp.csr_matrix((rv.cpu().numpy(), ri.to(torch.int32).cpu().numpy(), rip.cpu().numpy()),
                            shape=(self.n_recv, x.shape[1]))
        out.has_sorted_indices = bool(getattr(x, "has_sorted_indices", False))
        return out

    def forward_strings(self, ids: np.ndarray) -> np.ndarray:
        """Route a per-row string column (e.g. entity ids): per-row codes into this rank's table of distinct
        values (one int64 all-to-all) plus, to each destination, the UTF-8 bytes of only the distinct values its
        rows use (two variable-size all-to-alls of lengths and bytes) — no object collectives, no table
        all-gather."""
        import pandas as pd
        P = _world()
        codes, uniq = pd.factorize(np.asarray(ids, dtype=object), sort=False)
        codes = codes.astype(np.int64)
        dest = np.empty(self.n_local, dtype=np.int64)
        dest[self.perm] = np.repeat(np.arange(P), self.send_counts)
        # distinct values needed per destination, renumbered per destination
        pair = dest * max(len(uniq), 1) + codes
        up, pinv = np.unique(pair, return_inverse=True)
        u_dest, u_code = up // max(len(uniq), 1), up % max(len(uniq), 1)
        first = np.searchsorted(u_dest, np.arange(P))
        local_code = pinv - first[dest]                       # index into the destination's table
        enc = [str(v).encode("utf-8") for v in uniq[u_code]]
        blen = np.array([len(b) for b in enc], dtype=np.int64)
        tab_counts = np.bincount(u_dest, minlength=P).tolist()
        byte_counts = [int(blen[a:b].sum()) for a, b in _ranges(tab_counts)]
        payload = np.frombuffer(b"".join(enc), dtype=np.uint8).copy() if enc else np.zeros(0, np.uint8)
        rc = self.forward(torch.from_numpy(local_code)).numpy()
        if is_dist():
            rlen, rtab = all_to_all_varlen(torch.from_numpy(blen), tab_counts, self.group)
            rbytes, _ = all_to_all_varlen(torch.from_numpy(payload), byte_counts, self.group)
            rlen, rbytes = rlen.cpu().numpy(), bytes(rbytes.cpu().numpy())
        else:
            rlen, rtab, rbytes = blen, tab_counts, bytes(payload)
        ends = np.cumsum(rlen)
        names = np.array([rbytes[e - l:e].decode("utf-8") for e, l in zip(ends, rlen)], dtype=object)
        tab_base = np.concatenate([[0], np.cumsum(rtab)[:-1]]).astype(np.int64)
        return names[tab_base[self.src_rank] + rc] if len(rc) else np.zeros(0, dtype=object)


def _ranges(counts: Sequence[int]):
    s = 0
    for c in counts:
        yield s, s + int(c)
        s += int(c)


def gather_strings(values: Sequence[str], group=None) -> List[str]:
    """All-gather a list of strings (object collective; used once per coordinate for entity-id names)."""
    if not is_dist():
        return list(values)
    out: List[Optional[list]] = [None] * _world()
    dist.all_gather_object(out, list(values), group=group)
    return [s for part in out for s in part]
