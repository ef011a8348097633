"""Entity-aligned row placement for multi-GPU GAME.

The reference keys every random-effect dataset by entity and re-partitions it with a shuffle
(``photon-api/.../data/RandomEffectDataSet.scala:68-88``, ``RandomEffectDataSetPartitioner.scala:113-147``); its
fixed effect reads the same rows wherever they happen to live (``FixedEffectDataSet.scala``). Here rows are
placed ONCE, at ingest, on the rank that owns their entity in the PRIMARY random-effect coordinate: every feature
shard, response, offset, weight, uid and id tag travels in the one all-to-all (C8) that entity sharding needs
anyway. The fixed effect is row-parallel and placement-agnostic (a data-parallel all-reduce of per-rank sums), so
it trains on the placed rows as they are, and the primary random-effect coordinate finds all of its rows local:
its per-update residual / score routing (C11 / C12) becomes the identity — no bytes move. Other random-effect
coordinates keep their :class:`~photon_ml_amd.parallel.sharding.RowRouter`.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from ..data.game_data import GameData
from .sharding import EntityPartitioner, RowRouter, entity_keys


@dataclass
class EntityPlacement:
    """Attached to placed data (``GameData.placement``): the random-effect type the rows follow and the partitioner
    that decided the owners (the primary coordinate must use the same one)."""
    re_type: str
    partitioner: EntityPartitioner
    rows_moved: int          # rows this rank sent to other ranks at ingest


def route_game_data(data: GameData, router: RowRouter, device) -> GameData:
    """Every per-row array of ``data`` through ``router`` (feature shards as device CSR on a GPU, scipy on the host;
    integer id tags as one all-to-all each, string ids / raw uids as codes + the distinct names)."""
    dev = torch.device(device)

    def fwd(a):
        return router.forward(torch.from_numpy(np.ascontiguousarray(a)).to(dev)).cpu().numpy()

    def fwd_ids(v):
        v = np.asarray(v)
        return fwd(v.astype(np.int64)) if v.dtype.kind in "iu" else router.forward_strings(v)

    shards = {}
    for sid, x in data.shards.items():
        shards[sid] = router.forward_csr_device(x, dev) if dev.type == "cuda" else router.forward_csr(
            x.to_scipy() if hasattr(x, "to_scipy") else x)
    tags = {k: fwd_ids(v) for k, v in data.id_tags.items()}
    raw = None if data.raw_uids is None else fwd_ids(data.raw_uids)
    return GameData(fwd(data.response), shards, tags, fwd(data.offsets), fwd(data.weights), fwd(data.uids), raw)


def place_rows_by_entity(data: GameData, re_type: str, device) -> GameData:
    """``data`` re-distributed so every row lives on the owner of its ``re_type`` entity (rows of one source rank
    keep their order; the owner holds the rows of source ranks 0, 1, ... in turn — exactly the order the entity
    router delivers, so the primary coordinate sees the same rows in the same order as with per-update routing).
    Collective: every rank calls it. The result carries ``placement`` (:class:`EntityPlacement`)."""
    from .dist import rank as _rank
    ids = np.asarray(data.id_tags[re_type])
    keys = entity_keys(ids, torch.device(device))
    part = EntityPartitioner.build_t(keys)
    router = RowRouter(part.owner_t(keys))
    del keys
    out = route_game_data(data, router, device)
    moved = int(sum(router.send_counts) - router.send_counts[_rank()])
    out.placement = EntityPlacement(re_type, part, moved)
    return out
