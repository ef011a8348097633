"""Mid-training checkpoint / resume (SURVEY §5 "Checkpoint / resume" — absent in the reference, which only
persists final models; Spark lineage recomputation was its only recovery).

* GAME coordinate descent: after every coordinate update the current GAME model, the sweep position
  (iteration, next coordinate), the best model so far with its evaluations and the history are written to
  ``<dir>/cd-state[-rank<r>].safetensors`` (atomic rename). ``CoordinateDescent.run(..., checkpointer=...)``
  resumes from the next coordinate: scores are recomputed from the restored model (one scoring pass), so no
  N-length arrays are stored.
* Legacy λ path: every finished (λ, model) is stored; a resumed run skips the λ values already trained and
  warm-starts from the last one.

Format: safetensors (tensors / numpy arrays only, nothing executable) + a JSON metadata string. Every rank of a
process group writes its own file (entity-sharded random effects differ per rank). ``format_version`` 2 stores
entity-id tables length-prefixed and the writer's world size; version-less files still load: those with a world
size are length-prefixed (builds that predate the version field), the others are sniffed (first format: ids joined
by newlines).
"""
from __future__ import annotations

import json
import os
from collections import OrderedDict
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ..constants import TaskType

FORMAT_VERSION = 2
log = __import__("logging").getLogger(__name__)


def _rank() -> int:
    from ..parallel.dist import rank
    return rank()


def _world() -> int:
    from ..parallel.dist import world_size
    return world_size()


def _strings_to_array(values) -> np.ndarray:
    """Length-prefixed UTF-8 strings: ``[n, len_0 .. len_{n-1}]`` as little-endian int64 bytes, then the data
    (ids may contain any character, including newlines)."""
    enc = [str(v).encode("utf-8") for v in values]
    head = np.array([len(enc)] + [len(b) for b in enc], dtype="<i8").tobytes()
    return np.frombuffer(head + b"".join(enc), dtype=np.uint8).copy()


def _is_length_prefixed(raw: bytes, n: int) -> bool:
    """True when ``raw`` parses as a length-prefixed table of exactly ``n`` ids (count header and lengths add up)."""
    if len(raw) < 8 + 8 * n or int(np.frombuffer(raw[:8], dtype="<i8")[0]) != n:
        return False
    lens = np.frombuffer(raw[8:8 + 8 * n], dtype="<i8")
    return bool((lens >= 0).all()) and 8 + 8 * n + int(lens.sum()) == len(raw)


def _array_to_strings(a: np.ndarray, n: int, version: Optional[int] = FORMAT_VERSION) -> np.ndarray:
    """Decode an entity-id table. ``version`` None = a file without ``format_version``: builds between the two
    formats already wrote length-prefixed tables without the version field, so the layout is sniffed (a table
    whose count header and lengths add up exactly is length-prefixed; otherwise newline-joined)."""
    raw = bytes(np.ascontiguousarray(a).tobytes())
    if version is None:
        version = 2 if _is_length_prefixed(raw, n) else 1
    if version < 2:     # first format: UTF-8 ids joined by newlines
        ids = raw.decode("utf-8").split("\n") if n else []
        if len(ids) != n:
            raise ValueError(f"checkpoint entity table holds {len(ids)} ids, metadata says {n}")
        return np.array(ids, dtype=object)
    count = int(np.frombuffer(raw[:8], dtype="<i8")[0]) if len(raw) >= 8 else -1
    if count != n:
        raise ValueError(f"checkpoint entity table holds {count} ids, metadata says {n}")
    lens = np.frombuffer(raw[8:8 + 8 * n], dtype="<i8")
    ends = 8 + 8 * n + np.cumsum(lens)
    if n and ends[-1] != len(raw):
        raise ValueError("checkpoint entity table is truncated or corrupt")
    starts = ends - lens
    return np.array([raw[s:e].decode("utf-8") for s, e in zip(starts, ends)], dtype=object)


def game_model_to_arrays(model, prefix: str) -> Tuple[Dict[str, np.ndarray], dict]:
    from ..models.game import FixedEffectModel, RandomEffectModel
    arrays, meta = {}, {"coordinates": []}
    for cid, m in model:
        key = f"{prefix}{cid}"
        if isinstance(m, FixedEffectModel):
            c = m.glm.coefficients
            arrays[key + ".means"] = c.means.detach().cpu().numpy().astype(np.float64)
            if c.variances is not None:
                arrays[key + ".variances"] = c.variances.detach().cpu().numpy().astype(np.float64)
            meta["coordinates"].append({"id": cid, "kind": "fixed", "shard": m.feature_shard_id,
                                        "task": m.task.value})
        elif isinstance(m, RandomEffectModel):
            arrays[key + ".keys"] = m.keys
            arrays[key + ".values"] = m.values
            if m.variances is not None:
                arrays[key + ".variances"] = m.variances
            arrays[key + ".entities"] = _strings_to_array(m.entity_ids)
            meta["coordinates"].append({"id": cid, "kind": "random", "shard": m.feature_shard_id,
                                        "re_type": m.random_effect_type, "task": m.task.value, "dim": m.dim,
                                        "n_entities": int(m.n_entities)})
        else:
            raise TypeError(type(m))
    return arrays, meta


def game_model_from_arrays(arrays: Dict[str, np.ndarray], meta: dict, prefix: str,
                           version: Optional[int] = FORMAT_VERSION):
    from ..models.game import FixedEffectModel, GameModel, RandomEffectModel
    from ..models.glm import Coefficients, model_for_task
    models = OrderedDict()
    for c in meta["coordinates"]:
        key = f"{prefix}{c['id']}"
        task = TaskType.parse(c["task"])
        if c["kind"] == "fixed":
            var = arrays.get(key + ".variances")
            coef = Coefficients(torch.from_numpy(arrays[key + ".means"].copy()),
                                None if var is None else torch.from_numpy(var.copy()))
            models[c["id"]] = FixedEffectModel(model_for_task(task, coef), c["shard"])
        else:
            ents = _array_to_strings(arrays[key + ".entities"], c["n_entities"], version)
            models[c["id"]] = RandomEffectModel(c["re_type"], c["shard"], task, ents, c["dim"],
                                                arrays[key + ".keys"], arrays[key + ".values"],
                                                arrays.get(key + ".variances"))
    return GameModel(models)


class Checkpointer:
    """Writes / reads one state file per rank under ``directory``."""

    def __init__(self, directory: str, name: str = "cd-state"):
        self.directory = directory
        self.name = name
        os.makedirs(directory, exist_ok=True)

    @property
    def path(self) -> str:
        r = _rank()
        return os.path.join(self.directory, f"{self.name}{'' if r == 0 else f'-rank{r}'}.safetensors")

    def save(self, arrays: Dict[str, np.ndarray], meta: dict):
        from safetensors.numpy import save_file
        tmp = self.path + ".tmp"
        arrays = {k: np.ascontiguousarray(v) for k, v in arrays.items()}
        if not arrays:
            arrays = {"_empty": np.zeros(1)}
        save_file(arrays, tmp, metadata={"meta": json.dumps(meta)})
        os.replace(tmp, self.path)

    def load(self) -> Optional[Tuple[Dict[str, np.ndarray], dict]]:
        if not os.path.exists(self.path):
            return None
        from safetensors import safe_open
        arrays = {}
        with safe_open(self.path, framework="numpy") as f:
            meta = json.loads(f.metadata()["meta"])
            for k in f.keys():
                arrays[k] = f.get_tensor(k)
        return arrays, meta

    def exists(self) -> bool:
        return os.path.exists(self.path)

    # ---- coordinate descent state
    def save_cd(self, model, iteration: int, next_coordinate: int, best_model, best_evals, history: List[dict],
                tag: str = ""):
        from ..sampling.samplers import seed_state
        arrays, meta = game_model_to_arrays(model, "model/")
        meta = {"model": meta, "iteration": iteration, "next": next_coordinate, "tag": tag,
                "history": history, "best_evals": best_evals, "world_size": _world(),
                "format_version": FORMAT_VERSION, "sampler_seed_state": seed_state()}
        if best_model is not None:
            ba, bm = game_model_to_arrays(best_model, "best/")
            arrays.update(ba)
            meta["best"] = bm
        self.save(arrays, meta)

    def load_cd(self):
        got = self.load()
        if got is None:
            return None
        arrays, meta = got
        # no format_version: either the first (newline) format or a length-prefixed build that predates the field
        # (those already recorded world_size); the id tables are sniffed per coordinate in that case
        version = int(meta["format_version"]) if "format_version" in meta else (2 if "world_size" in meta else None)
        if version is not None and version > FORMAT_VERSION:
            raise RuntimeError(f"checkpoint {self.path} has format version {version}; this build reads <= "
                               f"{FORMAT_VERSION}")
        if "world_size" not in meta:
            log.warning("checkpoint %s does not record its world size (first format): resuming assumes the same "
                        "number of ranks wrote it", self.path)
        elif meta["world_size"] != _world():
            # entity-sharded random effects: each rank's file holds the entities that rank owned
            raise RuntimeError(f"checkpoint {self.path} was written by {meta['world_size']} ranks, "
                               f"this run has {_world()}: resume with the same world size")
        if "sampler_seed_state" in meta:
            # down-sampling seeds continue where the interrupted run stopped (bitwise resume with down-sampling)
            from ..sampling.samplers import set_seed_state
            set_seed_state(meta["sampler_seed_state"])
        model = game_model_from_arrays(arrays, meta["model"], "model/", version)
        best = game_model_from_arrays(arrays, meta["best"], "best/", version) if "best" in meta else None
        return {"model": model, "iteration": meta["iteration"], "next": meta["next"], "best_model": best,
                "best_evals": meta.get("best_evals"), "history": meta.get("history", []), "tag": meta.get("tag")}

    # ---- optimizer state (mid-solve checkpoint of one GLM / fixed-effect optimisation)
    def save_optimizer(self, optimizer, tag: str = ""):
        """Serialise ``optimizer.state_dict()``: tensors -> safetensors arrays (fp64, host copies), scalars and
        structure -> JSON metadata. Resuming with :meth:`load_optimizer` continues bitwise-identically."""
        arrays: Dict[str, np.ndarray] = {}

        def enc(v, key):
            import torch
            if isinstance(v, torch.Tensor):
                arrays[key] = v.detach().cpu().numpy()
                return {"__t": key, "device": str(v.device)}
            if isinstance(v, dict):
                return {k: enc(x, f"{key}/{k}") for k, x in v.items()}
            if isinstance(v, (list, tuple)):
                return {"__l": [enc(x, f"{key}/{i}") for i, x in enumerate(v)]}
            return v

        meta = {"optimizer": enc(optimizer.state_dict(), "opt"), "tag": tag}
        self.save(arrays, meta)

    def load_optimizer(self, optimizer, device=None) -> bool:
        """Restore into ``optimizer``; returns False when there is no checkpoint."""
        got = self.load()
        if got is None:
            return False
        arrays, meta = got
        import torch

        def dec(v):
            if isinstance(v, dict) and "__t" in v:
                return torch.from_numpy(arrays[v["__t"]].copy()).to(device or v["device"])
            if isinstance(v, dict) and "__l" in v:
                return [dec(x) for x in v["__l"]]
            if isinstance(v, dict):
                return {k: dec(x) for k, x in v.items()}
            return v

        optimizer.load_state_dict(dec(meta["optimizer"]))
        return True

