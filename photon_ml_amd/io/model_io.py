"""GAME / GLM model persistence in the reference's on-disk layout (Avro coefficients + JSON metadata).

Reference: ``photon-client/.../data/avro/ModelProcessingUtils.scala:63-684`` and ``AvroUtils.scala:185-430``:

    <root>/model-metadata.json                   {"modelType": <TaskType>, "optimizationConfigurations": {...}}
    <root>/fixed-effect/<coordinateId>/id-info   featureShardId
    <root>/fixed-effect/<coordinateId>/coefficients/part-00000.avro     one BayesianLinearModelAvro, modelId
                                                                         "fixed-effect"
    <root>/random-effect/<coordinateId>/id-info  randomEffectType \\n featureShardId
    <root>/random-effect/<coordinateId>/coefficients/part-XXXXX.avro    one record per entity (modelId = entity id)

Coefficients are written as NameTermValue triples for |value| > 1e-4, sorted by |value| descending; variances (when
present) use the same features. The loader only regex-reads ``modelType`` from the metadata (like the reference),
accepts the reference's model class FQCNs, and (unlike the reference, Appendix C.11) keeps variances.
"""
from __future__ import annotations

import json
import os
import re
from collections import OrderedDict
from typing import Dict, Optional

import numpy as np
import torch

from ..constants import MODEL_SPARSITY_THRESHOLD, TaskType, split_feature_key, feature_key
from ..models.game import FixedEffectModel, GameModel, RandomEffectModel
from ..models.glm import FQCN, LOSS_FQCN, Coefficients, model_for_task, task_from_model_class
from .avro import BAYESIAN_LINEAR_MODEL, read_records, write_records, avro_files
from .index_map import IndexMap

# random-effect models are written by the native encoder (write_linear_models); 0: per-record Python dictionaries
NATIVE_MODEL_WRITER = os.environ.get("PML_NATIVE_MODEL_WRITER", "1") != "0"
# Avro codec of the model files. The reference saves them through Hadoop's AvroOutputFormat without output
# compression configured (AvroUtils.saveAsAvro), i.e. uncompressed; "deflate" / "snappy" are available (a 3.5 GB
# random-effect model took ~50 s to deflate on 16 cores, its values barely compress).
MODEL_CODEC = os.environ.get("PML_MODEL_CODEC", "null")
# uncompressed bytes per Avro block (Avro's own writers cut blocks at a sync interval of this order)
BLOCK_BYTES = 1 << 20

FIXED_EFFECT = "fixed-effect"
RANDOM_EFFECT = "random-effect"
ID_INFO = "id-info"
COEFFICIENTS = "coefficients"
METADATA = "model-metadata.json"


def _ntv(values: np.ndarray, idx: np.ndarray, index_map: IndexMap):
    keep = np.abs(values) > MODEL_SPARSITY_THRESHOLD
    idx, values = idx[keep], values[keep]
    order = np.argsort(-np.abs(values), kind="stable")
    out = []
    for i, v in zip(idx[order], values[order]):
        key = index_map.get_feature_name(int(i))
        if key is None:
            raise KeyError(f"Feature index {i} not found in the feature map")
        n, t = split_feature_key(key)
        out.append({"name": n, "term": t, "value": float(v)})
    return out, idx[order]


def _feature_names(index_map: IndexMap, idx: np.ndarray):
    """Feature keys of the indices ``idx`` (batched where the map supports it)."""
    if hasattr(index_map, "get_feature_names"):
        names = index_map.get_feature_names(idx)
    elif hasattr(index_map, "index_to_key"):
        tab = index_map.index_to_key
        names = [tab[i] if 0 <= i < len(tab) else None for i in idx.tolist()]
    else:
        names = [index_map.get_feature_name(int(i)) for i in idx]
    for i, n in zip(idx, names):
        if n is None:
            raise KeyError(f"Feature index {i} not found in the feature map")
    return names


def block_records(n_models: int, n_kept: int, with_variances: bool) -> int:
    """Models per Avro block for ~BLOCK_BYTES uncompressed blocks (an estimate from the kept-coefficient count:
    ~24 bytes per name/term/value triple), so a file of large per-entity models still splits into many blocks that
    encode in parallel. The same for the native and the Python writers (same bytes)."""
    per = 96 + 24 * (2 if with_variances else 1) * n_kept / max(n_models, 1)
    return int(min(4096, max(1, BLOCK_BYTES // per)))


def write_linear_models(path: str, model_ids, ptr: np.ndarray, feat: np.ndarray, means: np.ndarray,
                        variances: Optional[np.ndarray], index_map: IndexMap, task: TaskType):
    """BayesianLinearModelAvro records of many models (model k = coefficients ``ptr[k]:ptr[k+1]`` at feature indices
    ``feat``) in one native call: the coefficient filter (|w| > MODEL_SPARSITY_THRESHOLD), the ordering by |w| and
    the Avro encoding + compression run in C++ over all cores; only the names of the features that occur are looked
    up. Same bytes as ``write_records`` of the ``glm_to_avro_record`` dictionaries (``tests/test_estimator_io.py``).
    Reference: ``photon-client/.../io/ModelProcessingUtils.scala`` (saveGameModelToHDFS)."""
    from .avro import native
    from ..constants import DELIMITER
    feat = np.ascontiguousarray(feat, dtype=np.int64)
    means = np.ascontiguousarray(means, dtype=np.float64)
    keep = np.abs(means) > MODEL_SPARSITY_THRESHOLD      # names only for coefficients that are written
    # distinct kept features and each coefficient's code by a marks table over the feature space (O(n); a sort /
    # binary search of 300M coefficients took most of a 3.5 GB model's save)
    dim = int(feat.max()) + 1 if len(feat) else 0
    seen = np.zeros(dim, dtype=bool)
    seen[feat[keep]] = True
    uniq = np.flatnonzero(seen)
    lut = np.zeros(dim, dtype=np.int64)
    lut[uniq] = np.arange(len(uniq), dtype=np.int64)
    code = lut[feat]
    code[~keep] = 0
    names = _feature_names(index_map, uniq) if len(uniq) else [""]
    blob = "\0".join(names).encode("utf-8")
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    native().write_linear_models(str(path), json.dumps(BAYESIAN_LINEAR_MODEL), [str(m) for m in model_ids],
                                 np.ascontiguousarray(ptr, dtype=np.int64), code.astype(np.int64),
                                 np.ascontiguousarray(means, dtype=np.float64),
                                 None if variances is None else np.ascontiguousarray(variances, dtype=np.float64),
                                 blob, FQCN[task], LOSS_FQCN.get(task), float(MODEL_SPARSITY_THRESHOLD), MODEL_CODEC,
                                 block_records(len(ptr) - 1, int(keep.sum()), variances is not None), DELIMITER)


def glm_to_avro_record(model_id: str, task: TaskType, means: np.ndarray, variances: Optional[np.ndarray],
                       index_map: IndexMap, idx: Optional[np.ndarray] = None) -> dict:
    idx = np.arange(len(means)) if idx is None else idx
    m, kept = _ntv(np.asarray(means, dtype=np.float64), np.asarray(idx), index_map)
    rec = {"modelId": model_id, "modelClass": FQCN[task], "means": m, "variances": None,
           "lossFunction": LOSS_FQCN.get(task)}
    if variances is not None:
        vmap = dict(zip(np.asarray(idx).tolist(), np.asarray(variances).tolist()))
        rec["variances"] = [{"name": e["name"], "term": e["term"], "value": float(vmap[int(i)])}
                            for e, i in zip(m, kept)]
    return rec


def avro_record_to_coefficients(rec: dict, index_map: IndexMap):
    means = np.zeros(index_map.feature_dimension)
    keys = [feature_key(e["name"], e.get("term") or "") for e in rec["means"]]
    idx = index_map.get_indices(keys) if keys else np.zeros(0, np.int64)
    vals = np.array([e["value"] for e in rec["means"]], dtype=np.float64)
    ok = idx >= 0
    means[idx[ok]] = vals[ok]
    variances = None
    if rec.get("variances"):
        variances = np.zeros(index_map.feature_dimension)
        vkeys = [feature_key(e["name"], e.get("term") or "") for e in rec["variances"]]
        vidx = index_map.get_indices(vkeys)
        vv = np.array([e["value"] for e in rec["variances"]])
        variances[vidx[vidx >= 0]] = vv[vidx >= 0]
    return means, variances


def opt_configs_to_json(configs) -> dict:
    if not configs:
        return {}
    return {cid: c.to_json() if hasattr(c, "to_json") else c for cid, c in configs.items()}


def save_game_model(model: GameModel, out_dir: str, index_maps: Dict[str, IndexMap], task=None,
                    opt_configs=None, re_file_limit: Optional[int] = None, entities_per_file: int = 100000):
    from ..parallel.dist import is_dist, rank
    task = TaskType.parse(task) if task is not None else model.task
    os.makedirs(out_dir, exist_ok=True)
    # under a process group: rank 0 writes metadata + (replicated) fixed effects; every rank writes the random-effect
    # entities it owns as its own part files (the reference saves RE RDD partitions in parallel the same way)
    sharded, r = is_dist(), rank()
    lead = r == 0
    if lead:
        with open(os.path.join(out_dir, METADATA), "w") as f:
            json.dump({"modelType": task.value, "optimizationConfigurations": opt_configs_to_json(opt_configs)}, f,
                      indent=2)
    for cid, m in model:
        if isinstance(m, FixedEffectModel) and not lead:
            continue
        if isinstance(m, FixedEffectModel):
            d = os.path.join(out_dir, FIXED_EFFECT, cid)
            os.makedirs(os.path.join(d, COEFFICIENTS), exist_ok=True)
            with open(os.path.join(d, ID_INFO), "w") as f:
                f.write(m.feature_shard_id + "\n")
            c = m.glm.coefficients
            means = c.means.cpu().numpy()
            var = None if c.variances is None else c.variances.cpu().numpy()
            path = os.path.join(d, COEFFICIENTS, "part-00000.avro")
            if NATIVE_MODEL_WRITER:
                write_linear_models(path, [FIXED_EFFECT], np.array([0, len(means)]), np.arange(len(means)), means,
                                    var, index_maps[m.feature_shard_id], task)
            else:
                rec = glm_to_avro_record(FIXED_EFFECT, task, means, var, index_maps[m.feature_shard_id])
                write_records(path, BAYESIAN_LINEAR_MODEL, [rec], codec=MODEL_CODEC, block_records=1)
        elif isinstance(m, RandomEffectModel):
            d = os.path.join(out_dir, RANDOM_EFFECT, cid)
            os.makedirs(os.path.join(d, COEFFICIENTS), exist_ok=True)
            if lead:
                with open(os.path.join(d, ID_INFO), "w") as f:
                    f.write(m.random_effect_type + "\n" + m.feature_shard_id + "\n")
            im = index_maps[m.feature_shard_id]
            keys, vals = m.keys, m.values
            ent = keys // m.dim
            feat = keys % m.dim
            bounds = np.searchsorted(ent, np.arange(m.n_entities + 1))
            present = np.nonzero(bounds[1:] > bounds[:-1])[0]          # entities with coefficients
            n_files = max(1, (len(present) + entities_per_file - 1) // entities_per_file)
            if re_file_limit is not None:
                n_files = max(1, min(n_files, re_file_limit))
            per = (len(present) + n_files - 1) // n_files if len(present) else 0
            prefix = f"part-r{r:05d}-" if sharded else "part-"
            for i in range(n_files):
                ents = present[i * per:(i + 1) * per]
                path = os.path.join(d, COEFFICIENTS, f"{prefix}{i:05d}.avro")
                if NATIVE_MODEL_WRITER:
                    # the entities' coefficient ranges are contiguous and in order: one slice per file
                    lo = bounds[ents[0]] if len(ents) else 0
                    hi = bounds[ents[-1] + 1] if len(ents) else 0
                    ptr = np.concatenate([bounds[ents], [hi]]) - lo if len(ents) else np.zeros(1, np.int64)
                    write_linear_models(path, [str(m.entity_ids[e]) for e in ents], ptr, feat[lo:hi], vals[lo:hi],
                                        None if m.variances is None else m.variances[lo:hi], im, task)
                    continue
                recs = [glm_to_avro_record(str(m.entity_ids[e]), task, vals[bounds[e]:bounds[e + 1]],
                                           None if m.variances is None else m.variances[bounds[e]:bounds[e + 1]],
                                           im, feat[bounds[e]:bounds[e + 1]]) for e in ents]
                write_records(path, BAYESIAN_LINEAR_MODEL, recs, codec=MODEL_CODEC,
                              block_records=block_records(len(recs), sum(len(r["means"]) for r in recs),
                                                          m.variances is not None))
        else:
            raise TypeError(f"unknown model type {type(m)}")


def load_model_task(model_dir: str) -> TaskType:
    p = os.path.join(model_dir, METADATA)
    if not os.path.exists(p):
        return TaskType.NONE
    txt = open(p).read()
    m = re.search(r'"modelType"\s*:\s*"(.+?)"', txt)
    if not m:
        raise RuntimeError(f"Couldn't find 'modelType' in metadata file: {p}")
    return TaskType.parse(m.group(1))


def load_game_model(model_dir: str, index_maps: Dict[str, IndexMap]) -> GameModel:
    task = load_model_task(model_dir)
    models = OrderedDict()
    fe_root = os.path.join(model_dir, FIXED_EFFECT)
    if os.path.isdir(fe_root):
        for cid in sorted(os.listdir(fe_root)):
            d = os.path.join(fe_root, cid)
            shard = open(os.path.join(d, ID_INFO)).read().split()[0]
            recs = []
            for fpath in avro_files(os.path.join(d, COEFFICIENTS)):
                recs.extend(read_records(fpath)[1])
            if not recs:
                raise ValueError(f"no coefficients in {d}")
            rec = recs[0]
            t = task if task != TaskType.NONE else task_from_model_class(rec["modelClass"])
            means, var = avro_record_to_coefficients(rec, index_maps[shard])
            glm = model_for_task(t, Coefficients(torch.from_numpy(means),
                                                 None if var is None else torch.from_numpy(var)))
            models[cid] = FixedEffectModel(glm, shard)
    re_root = os.path.join(model_dir, RANDOM_EFFECT)
    if os.path.isdir(re_root):
        for cid in sorted(os.listdir(re_root)):
            d = os.path.join(re_root, cid)
            info = open(os.path.join(d, ID_INFO)).read().split()
            re_type, shard = info[0], info[1]
            im = index_maps[shard]
            recs = []
            for fpath in avro_files(os.path.join(d, COEFFICIENTS)):
                recs.extend(read_records(fpath)[1])
            ids = np.array(sorted(str(r["modelId"]) for r in recs), dtype=object)
            ids_s = ids.astype(str)
            pos = {e: i for i, e in enumerate(ids_s)}
            keys, vals, vars_ = [], [], []
            t = task
            for r in recs:
                if t == TaskType.NONE:
                    t = task_from_model_class(r["modelClass"])
                means, var = avro_record_to_coefficients(r, im)
                nz = np.nonzero(means)[0]
                e = pos[str(r["modelId"])]
                keys.append(e * im.feature_dimension + nz)
                vals.append(means[nz])
                if var is not None:
                    vars_.append(var[nz])
            models[cid] = RandomEffectModel(re_type, shard, t, ids_s, im.feature_dimension,
                                            np.concatenate(keys) if keys else np.zeros(0, np.int64),
                                            np.concatenate(vals) if vals else np.zeros(0),
                                            np.concatenate(vars_) if vars_ and len(vars_) == len(vals) else None)
    if not models:
        raise ValueError(f"no model found under {model_dir}")
    return GameModel(models)


def write_text_models(models, index_map: IndexMap, path: str):
    """Legacy Driver text model output: ``name\\tterm\\tvalue\\tlambda`` per line, sorted by value descending
    (``photon-client/.../util/IOUtils.scala:236-280``). ``models`` = [(lambda, GLM)]."""
    os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
    with open(path, "w") as f:
        for lam, glm in models:
            w = glm.coefficients.means.cpu().numpy()
            for i in np.argsort(-w, kind="stable"):
                n, t = split_feature_key(index_map.get_feature_name(int(i)) or str(i))
                f.write(f"{n}\t{t}\t{w[i]}\t{lam}\n")
