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
import os
import time
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


def _lsr(t: torch.Tensor, k: int) -> torch.Tensor:
    """Logical right shift of int64 tensors (torch's >> is arithmetic)."""
    return (t >> k) & ((1 << (64 - k)) - 1)


_HM1 = int(np.uint64(0xBF58476D1CE4E5B9).view(np.int64))
_HM2 = int(np.uint64(0x94D049BB133111EB).view(np.int64))


def entity_keys(ids, device=None) -> torch.Tensor:
    """:func:`stable_hash64` of the entity ids as an int64 tensor on ``device``. Integer ids are hashed ON the
    device (pandas' int64 hash is a splitmix64 finaliser; bitwise identical, so ownership does not depend on the
    path); string ids go through pandas on the host once."""
    dev = torch.device(device) if device is not None else torch.device("cpu")
    if isinstance(ids, torch.Tensor):
        t = ids.to(dev, torch.int64)
    else:
        a = np.asarray(ids)
        if a.dtype.kind not in "iu":
            return torch.from_numpy(stable_hash64(a)).to(dev)
        t = torch.from_numpy(np.ascontiguousarray(a.astype(np.int64, copy=False))).to(dev)
    t = t ^ _lsr(t, 30)
    t = t * _HM1
    t = t ^ _lsr(t, 27)
    t = t * _HM2
    return t ^ _lsr(t, 31)


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
        return self.owner_t(torch.from_numpy(np.asarray(keys, dtype=np.int64))).numpy()

    def owner_t(self, keys: torch.Tensor) -> torch.Tensor:
        """Owning rank of each key, computed where ``keys`` live (hash = key as uint64 mod n_parts, the bin-packed
        top entities from their table)."""
        keys = keys.to(torch.int64)
        P = self.n_parts
        out = torch.where(keys < 0, (keys.remainder(P) + (1 << 64) % P) % P, keys.remainder(P))
        if len(self.top_keys):
            tk = self._top_on(keys.device)
            pos = torch.searchsorted(tk[0], keys).clamp(max=tk[0].numel() - 1)
            hit = tk[0][pos] == keys
            out = torch.where(hit, tk[1][pos], out)
        return out

    def _top_on(self, device):
        cache = self.__dict__.setdefault("_top_cache", {})
        key = str(device)
        if key not in cache:
            cache[key] = (torch.from_numpy(self.top_keys).to(device), torch.from_numpy(self.top_owner).to(device))
        return cache[key]

    @staticmethod
    def build(local_keys: np.ndarray, group=None, top_k: int = TOP_ENTITIES) -> "EntityPartitioner":
        """All-gather per-rank (key, count) histograms (C9) and build the same partitioner everywhere."""
        return EntityPartitioner.build_t(torch.from_numpy(np.asarray(local_keys, dtype=np.int64)), group, top_k)

    @staticmethod
    def build_t(local_keys: torch.Tensor, group=None, top_k: int = TOP_ENTITIES) -> "EntityPartitioner":
        """:meth:`build` with the histograms formed where ``local_keys`` live (the GPU under RCCL: unique +
        counts, the gathered histograms' merge and the top-k selection are device sorts); only the top_k
        (key, count) pairs reach the host for the bin packing."""
        uk, cnt = torch.unique(local_keys.to(torch.int64), sorted=True, return_counts=True)
        keys = torch.cat(all_gather_varlen(uk, group))
        counts = torch.cat(all_gather_varlen(cnt.to(torch.int64), group))
        gk, inv = torch.unique(keys, sorted=True, return_inverse=True)
        gc = torch.zeros(gk.numel(), dtype=torch.int64, device=gk.device).index_add_(0, inv, counts)
        # count descending, key ascending (gk is ascending and the sort is stable) -- as np.lexsort((keys, -counts))
        top = torch.sort(-gc, stable=True).indices[:top_k]
        return EntityPartitioner(gk[top].cpu().numpy(), gc[top].cpu().numpy(), _world(), top_k)


class _PhaseClock:
    """Accumulates wall seconds per named phase into ``times`` (no-op when None); synchronises the device the
    phase ran on first, so a phase's asynchronous kernels are charged to it."""

    def __init__(self, times: Optional[dict], dev):
        self.times, self.dev = times, torch.device(dev)
        self.t = time.perf_counter()
        if times is not None:
            self._sync(self.dev)
            self.t = time.perf_counter()

    @staticmethod
    def _sync(dev):
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    def __call__(self, name: str, dev=None):
        if self.times is None:
            return
        self._sync(torch.device(dev) if dev is not None else self.dev)
        now = time.perf_counter()
        self.times[name] = self.times.get(name, 0.0) + now - self.t
        self.t = now


# largest RCCL all-to-all per call and rank (see RowRouter._a2a_device)
A2A_MAX_BYTES = int(os.environ.get("PML_A2A_MAX_BYTES", str(1 << 30)))


class RowRouter:
    """Fixed permutation between this rank's sample rows and the rows it owns after routing by ``dest``.

    ``forward(v)``: local sample order -> concatenation over source ranks of the rows sent here (owner order);
    ``backward(u)``: the inverse (owner order -> local sample order). Both are one ``all_to_all_single``.

    Vectors stay where they are: the permutation is cached on each device it is used on, and under RCCL (``nccl``
    backend) the all-to-all runs directly on device tensors — an RE update moves its N-length score vectors
    GPU to GPU over xGMI with no host staging (C11/C12). Only the gloo backend (CPU rehearsals) stages through host
    memory, because gloo collectives take CPU tensors.
    """

    def __init__(self, dest, group=None):
        self.group = group
        P = _world()
        self._perm_on = {}
        if isinstance(dest, torch.Tensor):       # device route: the permutation is a device sort
            dest = dest.to(torch.int64)
            perm_t = torch.argsort(dest, stable=True)
            self._perm_on[str(perm_t.device)] = perm_t
            self.perm = perm_t.cpu().numpy()
            self.send_counts = torch.bincount(dest, minlength=P).tolist()
            self.n_local = int(dest.numel())
        else:
            dest = np.asarray(dest, dtype=np.int64)
            self.n_local = len(dest)
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
        if dev.type == "cuda":
            return self._a2a_device(send.to(dev).contiguous(), sc, rc, tail).to(send.device), rc
        if len(sc) == 1:
            return send, rc                 # one host-staged rank: the self segment is the whole buffer
        # host-staged backend (gloo): the segment this rank keeps never leaves its device; only the others
        # are staged through the host and exchanged
        me = _rank()
        so, ro = int(sum(sc[:me])), int(sum(rc[:me]))
        keep = send[so:so + sc[me]]
        sc2, rc2 = list(sc), list(rc)
        sc2[me] = rc2[me] = 0
        send2 = torch.cat([send[:so], send[so + sc[me]:]]).to(dev).contiguous()
        got = torch.empty((sum(rc2),) + tail, dtype=send.dtype, device=dev)
        dist.all_to_all_single(got, send2, rc2, sc2, group=self.group)
        got = got.to(send.device)
        return torch.cat([got[:ro], keep, got[ro:]]), rc

    def _a2a_device(self, send: torch.Tensor, sc: List[int], rc: List[int], tail) -> torch.Tensor:
        """RCCL all-to-all of device buffers in rounds of at most ``A2A_MAX_BYTES`` per rank: a single
        ``all_to_all_single`` over a multi-GB buffer (the 1.2G-entry random-effect shard of GAME config 5 is 5-10 GB
        per array) was measured to leave the tail of the output unwritten (a one-rank RCCL group, round 6:
        ``profiles/rccl_a2a_chunking_r6.md``). Every rank runs the same number of rounds (one max all-reduce);
        in round k each peer segment contributes its k-th of that many equal slices, so sender and receiver agree
        on every slice size from the segment length alone."""
        from .dist import all_reduce_scalar
        row_bytes = send.element_size() * int(np.prod(tail)) if tail else send.element_size()
        out = torch.empty((sum(rc),) + tuple(tail), dtype=send.dtype, device=send.device)
        need = max(sum(sc), sum(rc)) * row_bytes
        rounds = int(all_reduce_scalar(float(-(-need // A2A_MAX_BYTES)), "max", group=self.group))
        if rounds <= 1:
            dist.all_to_all_single(out, send, rc, sc, group=self.group)
            return out

        def slices(counts, k):
            offs = np.concatenate([[0], np.cumsum(counts)])
            cs = [-(-c // rounds) for c in counts]
            return [(int(offs[p] + min(k * cs[p], counts[p])), int(offs[p] + min((k + 1) * cs[p], counts[p])))
                    for p in range(len(counts))]
        for k in range(rounds):
            ss, rs = slices(sc, k), slices(rc, k)
            part = torch.cat([send[a:b] for a, b in ss]) if ss else send[:0]
            got = torch.empty((sum(b - a for a, b in rs),) + tuple(tail), dtype=send.dtype, device=send.device)
            dist.all_to_all_single(got, part, [b - a for a, b in rs], [b - a for a, b in ss], group=self.group)
            o = 0
            for a, b in rs:
                out[a:b] = got[o:o + b - a]
                o += b - a
            del part, got
        return out

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

    def forward_csr_device(self, x, device, times: Optional[dict] = None) -> "DeviceCSR":
        """Route sparse rows and KEEP them on ``device`` (a :class:`DeviceCSR`): row lengths, column indices and
        values each one all-to-all of device tensors under RCCL, the entry permutation a device gather — no scipy
        and no host copy of the routed rows (they go straight to the device random-effect build). ``times``:
        seconds of the phases (conversion to tensors, entry permutation, collectives, assembly), accumulated."""
        from ..data.matrix import DeviceCSR
        dev = torch.device(device)
        # the entry permutation runs on the target device whenever it is a GPU (also under a host-staged
        # backend: a device gather, then only the outgoing segments cross the host in _a2a)
        cdev = dev if dev.type == "cuda" else comm_device(self.group)
        clock = _PhaseClock(times, cdev)
        if isinstance(x, DeviceCSR):
            indptr, x_ind, x_val = x.indptr.to(cdev), x.indices.to(cdev), x.data.to(cdev)
        else:
            x = x.tocsr()
            indptr = torch.from_numpy(x.indptr.astype(np.int64)).to(cdev)
            x_ind = torch.from_numpy(x.indices).to(cdev)
            x_val = torch.from_numpy(x.data).to(cdev, torch.float64)
        clock("csr_convert")
        lens = indptr[1:] - indptr[:-1]
        perm = self.perm_on(cdev)
        ol = lens[perm]
        tot = int(ol.sum())
        start = torch.cumsum(ol, 0) - ol
        ent = torch.repeat_interleave(indptr[:-1][perm] - start, ol, output_size=tot) + torch.arange(tot, device=cdev)
        ri = x_ind[ent].to(torch.int32)
        rv = x_val[ent]
        del ent, x_ind, x_val
        P = len(self.send_counts)
        seg = torch.repeat_interleave(torch.arange(P, device=cdev),
                                      torch.tensor(self.send_counts, dtype=torch.int64, device=cdev),
                                      output_size=perm.numel())
        nnz_send = torch.zeros(P, dtype=torch.int64, device=cdev).index_add_(0, seg, ol).tolist()
        clock("csr_permute")
        rl = self.forward(lens)
        rseg = torch.repeat_interleave(torch.arange(P, device=cdev),
                                       torch.tensor(self.recv_counts, dtype=torch.int64, device=cdev),
                                       output_size=rl.numel())
        nnz_recv = torch.zeros(P, dtype=torch.int64, device=cdev).index_add_(0, rseg, rl).tolist()
        if is_dist():
            ri, _ = self._a2a(ri, nnz_send, nnz_recv)
            rv, _ = self._a2a(rv, nnz_send, nnz_recv)
        clock("csr_collective")
        rip = torch.zeros(rl.numel() + 1, dtype=torch.int64, device=cdev)
        torch.cumsum(rl, 0, out=rip[1:])
        out = DeviceCSR(rip.to(dev), ri.to(dev), rv.to(dev), (self.n_recv, x.shape[1]),
                        bool(getattr(x, "has_sorted_indices", False)))
        clock("csr_assemble", dev)
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
