"""GAME dataset: samples aligned by position with several feature shards and id tags.

Reference: ``GameDatum`` (``photon-lib/.../data/GameDatum.scala:38-69``: response, optional offset/weight, map of
feature-shard vectors, id-tag map) and the DataFrame conversion ``photon-api/.../data/GameConverters.scala``
(unique sample id = ``zipWithIndex``). Instead of an RDD of per-sample objects, the dataset is columnar: every
array is indexed by the sample position, so scores/offsets of different coordinates combine elementwise (the
reference's full-outer-join score algebra disappears).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Optional

import numpy as np
import scipy.sparse as sp

from .matrix import LabeledData, as_csr


@dataclass
class GameData:
    response: np.ndarray
    shards: Dict[str, sp.csr_matrix]
    id_tags: Dict[str, np.ndarray] = field(default_factory=dict)
    offsets: Optional[np.ndarray] = None
    weights: Optional[np.ndarray] = None
    uids: Optional[np.ndarray] = None
    raw_uids: Optional[np.ndarray] = None  # original (string) uids from the input records, for score output
    # id tag -> (codes, distinct values, the tag array they encode): the reader's factorisation of a string id tag,
    # reused by the random-effect build instead of a sort of every row's string (valid only for that very array)
    id_factors: Optional[Dict[str, tuple]] = None

    def __post_init__(self):
        n = len(self.response)
        self.response = np.asarray(self.response, dtype=np.float64)
        self.offsets = np.zeros(n) if self.offsets is None else np.asarray(self.offsets, np.float64)
        self.weights = np.ones(n) if self.weights is None else np.asarray(self.weights, np.float64)
        self.uids = np.arange(n, dtype=np.int64) if self.uids is None else np.asarray(self.uids, np.int64)
        self.shards = {k: as_csr(v) for k, v in self.shards.items()}
        for k, v in self.shards.items():
            if v.shape[0] != n:
                raise ValueError(f"shard {k} has {v.shape[0]} rows, expected {n}")
        self.id_tags = {k: np.asarray(v) for k, v in self.id_tags.items()}

    @property
    def n_rows(self) -> int:
        return len(self.response)

    def shard(self, shard_id: str) -> sp.csr_matrix:
        if shard_id not in self.shards:
            raise KeyError(f"feature shard {shard_id} not present (have {sorted(self.shards)})")
        return self.shards[shard_id]

    def prefetch_shard(self, shard_id: str, device) -> bool:
        """Start copying the host CSR shard ``shard_id`` to ``device`` (int64 row pointers, the column indices, fp64
        values) on a side stream from a background thread, so the copy overlaps the GPU work queued before the
        shard's consumer runs (the random-effect build after the fixed-effect layout: the copy is a PCIe transfer,
        the layout build is device work). The copy starts once the next tiled build has uploaded its own shard
        (``ops.device.H2D_GATE``), so the two copies do not share the host link. :meth:`take_prefetched` hands the
        arrays over. False when there is nothing to do (no GPU, not a host CSR, already started)."""
        import threading
        import torch
        dev = torch.device(device)
        pre = self.__dict__.setdefault("_prefetch", {})
        x = self.shards.get(shard_id)
        if dev.type != "cuda" or shard_id in pre or not isinstance(x, sp.csr_matrix):
            return False
        side = torch.cuda.Stream(dev)
        out = {}
        from ..ops.device import H2D_GATE
        gate = H2D_GATE
        gate.clear()                 # set by the next tiled build's upload (or by take_prefetched)

        def run():
            gate.wait(timeout=30.0)
            try:
                with torch.cuda.device(dev), torch.cuda.stream(side):
                    out["arrays"] = (torch.from_numpy(x.indptr.astype(np.int64)).to(dev),
                                     torch.from_numpy(x.indices).to(dev),
                                     torch.from_numpy(x.data).to(dev, torch.float64))
                side.synchronize()
            except BaseException as e:       # surfaced by take_prefetched
                out["error"] = e

        th = threading.Thread(target=run, name=f"prefetch-{shard_id}", daemon=True)
        th.start()
        pre[shard_id] = (x, th, out, side)
        return True

    def take_prefetched(self, shard_id: str, x) -> Optional[tuple]:
        """The device arrays ``(indptr int64, indices, values fp64)`` of a shard started by :meth:`prefetch_shard`,
        if it was started for this very matrix ``x`` (waits for the copy); None otherwise. Hands them over once."""
        pre = self.__dict__.get("_prefetch", {}).pop(shard_id, None)
        if pre is None:
            return None
        src, th, out, side = pre
        from ..ops.device import H2D_GATE
        H2D_GATE.set()               # no upload to wait for any more: copy now if not yet started
        th.join()
        if "error" in out:
            raise out["error"]
        if src is not x:
            return None
        import torch
        arrays = out["arrays"]
        for t in arrays:
            t.record_stream(torch.cuda.current_stream(t.device))     # allocated on the side stream, used here
        return arrays

    def labeled(self, shard_id: str, offsets: Optional[np.ndarray] = None) -> LabeledData:
        return LabeledData(self.shard(shard_id), self.response, self.offsets if offsets is None else offsets,
                           self.weights, self.uids)

    def subset(self, rows) -> "GameData":
        rows = np.asarray(rows)
        return GameData(self.response[rows], {k: v[rows] for k, v in self.shards.items()},
                        {k: v[rows] for k, v in self.id_tags.items()}, self.offsets[rows], self.weights[rows],
                        self.uids[rows], None if self.raw_uids is None else self.raw_uids[rows])


def generate_game_data(n_rows: int = 2000, n_users: int = 50, n_items: int = 30, d_global: int = 20,
                       d_user: int = 6, d_item: int = 6, task: str = "LINEAR_REGRESSION", seed: int = 11,
                       noise: float = 0.1):
    """Synthetic mixed-effect data: y = x_g.w_g + x_u.w_user[u] + x_i.w_item[i] (+ noise / logistic link).

    Shards: ``global`` (d_global incl. intercept), ``user`` (d_user incl. intercept), ``item`` (d_item incl.
    intercept); id tags ``userId`` and ``itemId``. Returns ``(GameData, truth)``.
    """
    rng = np.random.default_rng(seed)
    users = rng.zipf(1.6, size=n_rows) % n_users
    items = rng.integers(0, n_items, size=n_rows)

    def shard(d, dens=0.5):
        x = sp.random(n_rows, d - 1, density=dens, format="csr", random_state=int(rng.integers(1 << 30)),
                      data_rvs=lambda k: rng.normal(size=k))
        return sp.hstack([x, np.ones((n_rows, 1))], format="csr")

    xg, xu, xi = shard(d_global), shard(d_user), shard(d_item)
    wg = rng.normal(size=d_global)
    wu = rng.normal(size=(n_users, d_user)) * 0.8
    wi = rng.normal(size=(n_items, d_item)) * 0.8
    z = xg @ wg + np.einsum("ij,ij->i", xu.toarray(), wu[users]) + np.einsum("ij,ij->i", xi.toarray(), wi[items])
    if task == "LOGISTIC_REGRESSION":
        y = (rng.random(n_rows) < 1 / (1 + np.exp(-z))).astype(float)
    elif task == "POISSON_REGRESSION":
        y = rng.poisson(np.exp(np.clip(z * 0.3, -10, 4))).astype(float)
    else:
        y = z + noise * rng.normal(size=n_rows)
    data = GameData(y, {"global": xg, "user": xu, "item": xi},
                    {"userId": np.array([f"u{u}" for u in users], dtype=object),
                     "itemId": np.array([f"i{i}" for i in items], dtype=object)})
    return data, {"global": wg, "user": wu, "item": wi}
