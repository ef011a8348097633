"""Synthetic data generators.

* :func:`generate_glm_data` — host (scipy) generator of binary, linear and Poisson data from a random ground
  truth (seeded, sparse features, intercept).
* :func:`draw_samples` — the reference's benign / outlier / invalid-feature / invalid-label test families
  (``photon-test-utils/.../SparkTestUtils.scala:85-308``).
* :func:`generate_device_shard` — ON-DEVICE generator of the benchmark shard (BASELINE config "logistic L-BFGS
  1B x 1M sparse", 125M rows per GPU at 8 GPUs). It writes the chunked CSR/CSC streams of
  :class:`~photon_ml_amd.ops.device.DeviceGLMData` directly in HBM without any host round trip of the entries.

  The structure is click-through-like hashed categorical data: the ``n_features - 1`` non-intercept columns are
  split into ``nnz_per_row - 1`` fields; each row takes exactly one column per field, drawn from a Zipf(s) law
  over the field's columns (hot features + long tail), with a value in [0.5, 1.5); the last column is the
  intercept (1.0 in every row). Labels are Bernoulli(sigmoid(x . w*)) for a random sparse ground truth w*.
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import scipy.sparse as sp
import torch

from ..constants import TaskType
from .matrix import LabeledData


# SparkTestUtils constants (photon-test-utils/.../SparkTestUtils.scala:310-316)
INLIER_PROBABILITY = 0.90
INLIER_STANDARD_DEVIATION = 1e-3
OUTLIER_STANDARD_DEVIATION = 1.0
SAMPLE_KINDS = ("benign", "outlier", "invalid_features", "invalid_labels")


def draw_samples(task, kind: str, seed: int, size: int, dimensionality: int,
                 desired_sparsity: float = 0.1) -> LabeledData:
    """Reference test-data families (``SparkTestUtils.scala:85-308, 320-873``): one row per sample, column 0 the
    label-correlated attribute, every other column present with probability ``desired_sparsity`` (the
    reference's negative-binomial skip-ahead coin toss).

    * ``benign``: dummy columns uniform in [-1, 1);
    * ``outlier``: dummy columns ``N(0, 1e-3)`` with probability 0.9, else +-1 (and, for linear regression, the
      attribute carries unit-variance noise);
    * ``invalid_features``: as outlier but the 10 % are NaN / +inf / -inf, plus NaN, +inf, -inf in the last three
      columns of every row;
    * ``invalid_labels``: benign features, labels drawn from {+inf, -inf, NaN}.

    Labels: binary classification 1/0 with probability 0.5 and a strictly separable attribute +-[0.1, 1);
    Poisson ``1 + 10 u`` with attribute ``log(label) / log(11)``; linear ``2u - 1`` (benign) or ``1 + u``.
    The RNG is numpy's (the reference's Well19937a streams are not reproduced), the families are."""
    task = TaskType.parse(task)
    if kind not in SAMPLE_KINDS:
        raise ValueError(f"unknown sample kind {kind!r}, expected one of {SAMPLE_KINDS}")
    rng = np.random.default_rng(5000 * seed)
    n, d = int(size), int(dimensionality)
    u = rng.random(n)
    binary = task in (TaskType.LOGISTIC_REGRESSION, TaskType.SMOOTHED_HINGE_LOSS_LINEAR_SVM)
    if kind == "invalid_labels":
        y = np.array([np.inf, -np.inf, np.nan])[rng.integers(0, 3, n)]
        x0 = 0.1 + 0.9 * u
    elif binary:
        y = (rng.random(n) <= 0.5).astype(np.float64)
        x0 = np.where(y == 1.0, 1.0, -1.0) * (0.1 + 0.9 * u)
    elif task == TaskType.POISSON_REGRESSION:
        y = 1.0 + 10.0 * u
        x0 = (np.log(y) + rng.normal(size=n) * INLIER_STANDARD_DEVIATION) / np.log(11.0)
    elif kind == "benign":
        y = 2.0 * u - 1.0
        x0 = y + rng.normal(size=n) * INLIER_STANDARD_DEVIATION
    else:
        y = 1.0 + u
        x0 = y - 1.0 + rng.normal(size=n) * OUTLIER_STANDARD_DEVIATION
    tail_end = d - 3 if kind == "invalid_features" else d
    mask = rng.random((n, max(tail_end - 1, 0))) < desired_sparsity
    rows, cols = np.nonzero(mask)
    cols = cols + 1
    k = rows.size
    if kind in ("benign", "invalid_labels"):
        vals = 2.0 * (rng.random(k) - 0.5)
    else:
        inlier = rng.random(k) < INLIER_PROBABILITY
        if kind == "outlier":
            bad = np.where(rng.random(k) < 0.5, 1.0, -1.0)
        else:
            bad = np.array([np.nan, np.inf, -np.inf])[rng.integers(0, 3, k)]
        vals = np.where(inlier, rng.normal(size=k) * INLIER_STANDARD_DEVIATION, bad)
    r_all = [np.arange(n), rows]
    c_all = [np.zeros(n, np.int64), cols]
    v_all = [x0, vals]
    if kind == "invalid_features":
        for j, v in zip((d - 3, d - 2, d - 1), (np.nan, np.inf, -np.inf)):
            r_all.append(np.arange(n))
            c_all.append(np.full(n, j))
            v_all.append(np.full(n, v))
    x = sp.csr_matrix((np.concatenate(v_all), (np.concatenate(r_all), np.concatenate(c_all))), shape=(n, d))
    x.sort_indices()
    return LabeledData(x, y)


def generate_glm_data(task, n_rows: int, n_features: int, density: float = 0.2, seed: int = 7,
                      intercept: bool = True, noise: float = 1e-3, kind: str = "benign"):
    """Host generator. Returns ``(LabeledData, w_true)``; the last column is the intercept when requested."""
    task = TaskType.parse(task)
    rng = np.random.default_rng(seed)
    d_feat = n_features - (1 if intercept else 0)
    x = sp.random(n_rows, d_feat, density=density, format="csr", random_state=seed,
                  data_rvs=lambda k: rng.uniform(-1, 1, size=k))
    if kind == "outlier":
        x.data *= np.where(rng.random(x.data.size) < 0.01, 1e3, 1.0)
    if intercept:
        x = sp.hstack([x, np.ones((n_rows, 1))], format="csr")
    w = rng.normal(size=n_features)
    z = x @ w
    if task == TaskType.LOGISTIC_REGRESSION or task == TaskType.SMOOTHED_HINGE_LOSS_LINEAR_SVM:
        y = (rng.random(n_rows) < 1.0 / (1.0 + np.exp(-z))).astype(np.float64)
    elif task == TaskType.POISSON_REGRESSION:
        w *= 0.2
        z = x @ w
        y = rng.poisson(np.exp(np.clip(z, -20, 5))).astype(np.float64)
    else:
        y = z + rng.normal(scale=noise, size=n_rows)
    if kind == "invalid":
        y[0] = np.nan
    return LabeledData(x, y), w


def zipf_cdf(n: int, s: float, device) -> torch.Tensor:
    k = torch.arange(1, n + 1, dtype=torch.float64, device=device)
    p = k.pow(-s)
    c = torch.cumsum(p, 0)
    return (c / c[-1]).to(torch.float32)


def generate_device_shard(n_rows: int, n_features: int, nnz_per_row: int, device="cuda", precision: str = "bf16",
                          seed: int = 1234567890, chunk_rows: int = 1 << 20, zipf_s: float = 1.1,
                          task=TaskType.LOGISTIC_REGRESSION, rank: int = 0, progress=None, layout: str = "auto"):
    """Generate a :class:`DeviceGLMData` directly in device memory (see module docstring)."""
    from ..ops.device import DeviceGLMData, SegChunk, VAL_DTYPE, resolve_layout
    from ..ops.tiled import TLFwdChunk, TLTChunk

    dev = torch.device(device)
    prec = {"bf16": 0, "f32": 1, "f64": 2}[precision]
    vdt = VAL_DTYPE[prec]
    n_fields = nnz_per_row - 1
    if n_fields < 1:
        raise ValueError("nnz_per_row must be >= 2 (intercept + >= 1 field)")
    fs = (n_features - 1) // n_fields
    if fs < 1:
        raise ValueError("not enough features for the requested nnz per row")
    layout = resolve_layout(layout, n_features, chunk_rows)
    cdf = zipf_cdf(fs, zipf_s, dev)
    field_base = (torch.arange(n_fields, device=dev, dtype=torch.int32) * fs)
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed + 7919 * rank)
    starts = list(range(0, n_rows, chunk_rows)) + [n_rows]
    k = nnz_per_row
    raw = []
    counts = torch.zeros(n_features, dtype=torch.int64, device=dev)
    for ci, (a, b) in enumerate(zip(starts[:-1], starts[1:])):
        m = b - a
        u = torch.rand((m, n_fields), generator=gen, device=dev)
        rank_ = torch.searchsorted(cdf, u).clamp_(max=fs - 1).to(torch.int32)
        del u
        idx = torch.empty((m, k), dtype=torch.int32, device=dev)
        idx[:, :n_fields] = rank_ + field_base
        idx[:, n_fields] = n_features - 1
        del rank_
        val = torch.empty((m, k), dtype=torch.float32, device=dev)
        val[:, :n_fields] = torch.rand((m, n_fields), generator=gen, device=dev) + 0.5
        val[:, n_fields] = 1.0
        idx = idx.reshape(-1)
        counts += torch.bincount(idx.to(torch.int64), minlength=n_features)
        raw.append((idx, val.to(vdt).reshape(-1)))
        if (m + 1) * k >= 2 ** 31:
            raise ValueError("chunk too large for int32 offsets: lower chunk_rows")
    # relabel features hottest-first (the forward kernel keeps the head of w in an LDS hot table); under a process
    # group the counts are summed first so every rank shares ONE feature order (gradient all-reduce buckets then
    # cover the same columns on every rank, see DistributedGLMData)
    import torch.distributed as dist
    from ..parallel.dist import is_dist
    if is_dist():
        cc = counts if dist.get_backend() == "nccl" else counts.cpu()
        dist.all_reduce(cc)
        counts = cc.to(dev)
    old_of_new = torch.argsort(counts, descending=True, stable=True)
    new_of_old = torch.empty_like(old_of_new)
    new_of_old[old_of_new] = torch.arange(n_features, device=dev)
    new_of_old32 = new_of_old.to(torch.int32)
    del counts
    csr, csc = [], []
    from ..ops.tiled import shard_t_config
    cbits, item_entries = shard_t_config(n_rows * k, n_rows, n_features, chunk_rows)
    for ci, ((a, b), (idx, val)) in enumerate(zip(zip(starts[:-1], starts[1:]), raw)):
        m = b - a
        idx = new_of_old32[idx.to(torch.int64)]
        if layout == "tiled":
            rp = torch.arange(0, (m + 1) * k, k, dtype=torch.int64, device=dev)
            col = idx.to(torch.int64)
            del idx
            csr.append(TLFwdChunk(rp, col, val, n_features))
            csc.append(TLTChunk(rp, col, val, n_features, chunk_rows, cbits=cbits, item_entries=item_entries))
            raw[ci] = None
            del col, val, rp
            if progress is not None:
                progress(ci + 1, len(starts) - 1)
            continue
        seg_ptr = np.arange(0, (m + 1) * k, k, dtype=np.int64).astype(np.int32)
        csr.append(SegChunk(seg_ptr, idx, val, dev, forward=True))
        # CSC of the chunk: stable sort by column -> rows stay ascending inside each column segment
        perm = torch.argsort(idx, stable=True)
        cidx = (perm // k).to(torch.int32)
        cval = val[perm]
        colptr = torch.zeros(n_features + 1, dtype=torch.int64, device=dev)
        colptr[1:] = torch.cumsum(torch.bincount(idx.to(torch.int64), minlength=n_features), 0)
        del perm
        csc.append(SegChunk(colptr.cpu().numpy().astype(np.int32), cidx, cval, dev))
        raw[ci] = None
        del cidx, cval, colptr, idx, val
        if progress is not None:
            progress(ci + 1, len(starts) - 1)
    y = torch.zeros(n_rows, dtype=torch.float32, device=dev)
    data = DeviceGLMData(csr, csc, starts, y, torch.zeros_like(y), torch.ones_like(y), n_features, precision, dev,
                         old_of_new)
    # labels from a sparse ground truth
    wgen = torch.Generator(device=dev)
    wgen.manual_seed(seed)
    w_true = torch.randn(n_features, generator=wgen, device=dev, dtype=torch.float64) * 0.3
    w_true[torch.rand(n_features, generator=wgen, device=dev) < 0.5] = 0.0
    w_true[-1] = -1.0
    z = data.margins(w_true)
    p = torch.sigmoid(z)
    task = TaskType.parse(task)
    if task == TaskType.LOGISTIC_REGRESSION:
        yy = (torch.rand(n_rows, generator=gen, device=dev, dtype=torch.float64) < p).to(torch.float32)
    elif task == TaskType.POISSON_REGRESSION:
        yy = torch.poisson(torch.exp(z.clamp(max=5.0)) * 0.2, generator=gen).to(torch.float32)
    else:
        yy = (z + 0.1 * torch.randn(n_rows, generator=gen, device=dev, dtype=torch.float64)).to(torch.float32)
    data.y.copy_(yy.to(data.vdt))
    return data, w_true


def _device_csr_to_host(counts: torch.Tensor, cols: torch.Tensor, vals: torch.Tensor, n_cols: int) -> sp.csr_matrix:
    """scipy CSR from per-row counts and the row-major (column, value) entries, all on the device."""
    indptr = torch.zeros(counts.numel() + 1, dtype=torch.int64, device=counts.device)
    torch.cumsum(counts, 0, out=indptr[1:])
    x = sp.csr_matrix((vals.cpu().numpy(), cols.to(torch.int32).cpu().numpy(), indptr.cpu().numpy()),
                      shape=(counts.numel(), n_cols))
    x.has_canonical_format = True          # strictly increasing columns per row (sorted, no duplicates)
    return x


def generate_game_bench_data_device(n_entities: int, rows_per_entity: int, re_dim: int = 100, re_nnz: int = 10,
                                    fe_dim: int = 100_000, fe_nnz: int = 30, re_vocab: int = 1 << 20, seed: int = 7,
                                    entity_offset: int = 0, task: str = "LOGISTIC_REGRESSION", pool: str = "random",
                                    int_ids: bool = False, sizes: str = "uniform", size_alpha: float = 1.3,
                                    max_rows: int = 20000, device="cuda", label_bias: float = 0.0,
                                    heavy_rows=()):
    """:func:`generate_game_bench_data` with every draw, sort and reduction on the device (torch), so benchmark
    GAME data of config-5 size (25M rows, 2.1G non-zeros per GPU) takes seconds instead of minutes of host numpy;
    only the finished CSR arrays cross to the host (the GameData container is host scipy). Same structure and
    distributions (entity size law, Zipf fixed-effect features, per-entity feature pools, ground-truth labels),
    different random streams; rows hold strictly increasing columns (canonical CSR, duplicates dropped).
    ``label_bias``: added to the ground-truth logit of logistic labels (e.g. -4: ~5 % positives, the imbalanced
    click data the reference's binary-classification down-sampler is meant for). ``heavy_rows``: row counts that
    replace the drawn sizes of the first entities (a heavy tail beyond ``max_rows``)."""
    from ..data.game_data import GameData
    dev = torch.device(device)
    gen = torch.Generator(device=dev)
    gen.manual_seed(int(seed))
    rnd = lambda *shape: torch.rand(shape, generator=gen, device=dev, dtype=torch.float64)
    if sizes == "powerlaw":
        if pool == "exact":
            raise ValueError("pool='exact' needs equal entity sizes")
        u = rnd(n_entities)
        target = n_entities * rows_per_entity
        xm = float(rows_per_entity) * (size_alpha - 1) / size_alpha
        for _ in range(30):          # scale so that the capped Pareto sizes have the requested mean
            cnt = torch.clamp(torch.ceil(xm * u ** (-1.0 / size_alpha)), max=max_rows).to(torch.int64)
            tot = int(cnt.sum())
            if abs(tot - target) <= 0.001 * target:
                break
            xm *= target / tot
    elif sizes == "uniform":
        cnt = torch.full((n_entities,), rows_per_entity, dtype=torch.int64, device=dev)
    else:
        raise ValueError(f"unknown entity size law {sizes!r}")
    if len(heavy_rows):
        cnt[:len(heavy_rows)] = torch.tensor([int(r) for r in heavy_rows], dtype=torch.int64, device=dev)
    n = int(cnt.sum())
    ent_sorted = torch.repeat_interleave(torch.arange(n_entities, device=dev), cnt, output_size=n)
    perm = torch.randperm(n, generator=gen, device=dev)
    ent = ent_sorted[perm]
    # ---- fixed-effect shard: fe_nnz Zipf(1.1) columns per row (duplicates dropped) + the intercept
    p = torch.arange(1, fe_dim, device=dev, dtype=torch.float64) ** -1.1
    cdf = torch.cumsum(p, 0)
    cdf /= cdf[-1].clone()
    fcol = torch.searchsorted(cdf, rnd(n, fe_nnz)).clamp_(max=fe_dim - 2)
    fcol, _ = torch.sort(fcol, dim=1)
    keep = torch.ones_like(fcol, dtype=torch.bool)
    keep[:, 1:] = fcol[:, 1:] != fcol[:, :-1]
    fval = rnd(n, fe_nnz) + 0.5
    fcol = torch.cat([fcol, torch.full((n, 1), fe_dim - 1, device=dev, dtype=fcol.dtype)], 1)
    fval = torch.cat([fval, torch.ones(n, 1, device=dev, dtype=torch.float64)], 1)
    keep = torch.cat([keep, torch.ones(n, 1, device=dev, dtype=torch.bool)], 1)
    xg = _device_csr_to_host(keep.sum(1), fcol[keep], fval[keep], fe_dim)
    wg = torch.randn(fe_dim, generator=gen, device=dev, dtype=torch.float64) * 0.2
    wg[-1] = -0.5
    zg = (fval * wg[fcol] * keep).sum(1)
    del fcol, fval, keep
    # ---- random-effect shard: pool slot k of entity e -> feature (hash(e) + k * stride) % re_vocab, + intercept
    if pool == "exact":
        if re_nnz > re_dim:
            raise ValueError("pool='exact' needs re_nnz <= re_dim")
        start = torch.zeros(n_entities, dtype=torch.int64, device=dev)
        torch.cumsum(cnt[:-1], 0, out=start[1:])
        within = perm - start[ent]          # row k = occurrence perm[k] - start[e] of its entity e
        slot = (within[:, None] * re_nnz + torch.arange(re_nnz, device=dev)[None, :]) % re_dim
        del within, start
    else:
        slot = torch.randint(0, re_dim, (n, re_nnz), generator=gen, device=dev)
    del ent_sorted, perm
    gid = ent + entity_offset
    base = (gid * 2654435761) % (re_vocab - 1)
    rcol = (base[:, None] + slot * 40503) % (re_vocab - 1)
    rval = torch.randn(n, re_nnz, generator=gen, device=dev, dtype=torch.float64)
    wgen = torch.Generator(device=dev)
    wgen.manual_seed(int(seed) + 1)
    w_slot = torch.randn(re_dim, generator=wgen, device=dev, dtype=torch.float64) * 0.5
    rcol, order = torch.sort(rcol, dim=1)
    slot = torch.gather(slot, 1, order)
    rval = torch.gather(rval, 1, order)
    del order
    rkeep = torch.ones_like(rcol, dtype=torch.bool)
    rkeep[:, 1:] = rcol[:, 1:] != rcol[:, :-1]
    zr = (rval * w_slot[slot] * rkeep).sum(1) + 0.3 * torch.sin(gid.to(torch.float64))
    del slot
    rcol = torch.cat([rcol, torch.full((n, 1), re_vocab - 1, device=dev, dtype=rcol.dtype)], 1)
    rval = torch.cat([rval, torch.ones(n, 1, device=dev, dtype=torch.float64)], 1)
    rkeep = torch.cat([rkeep, torch.ones(n, 1, device=dev, dtype=torch.bool)], 1)
    xr = _device_csr_to_host(rkeep.sum(1), rcol[rkeep], rval[rkeep], re_vocab)
    del rcol, rval, rkeep
    z = zg + zr
    task = TaskType.parse(task)
    if task == TaskType.LOGISTIC_REGRESSION:
        y = (rnd(n) < torch.sigmoid(z + label_bias)).to(torch.float64)
    elif task == TaskType.POISSON_REGRESSION:
        y = torch.poisson(torch.exp(torch.clamp(z * 0.3, -10, 3)), generator=gen)
    else:
        y = z + 0.1 * torch.randn(n, generator=gen, device=dev, dtype=torch.float64)
    gid_h = gid.cpu().numpy()
    ids = gid_h.copy() if int_ids else np.char.add("e", gid_h.astype(str)).astype(object)
    return GameData(y.cpu().numpy(), {"global": xg, "entity": xr}, {"entityId": ids})


def generate_game_bench_data(n_entities: int, rows_per_entity: int, re_dim: int = 100, re_nnz: int = 10,
                             fe_dim: int = 100_000, fe_nnz: int = 30, re_vocab: int = 1 << 20, seed: int = 7,
                             entity_offset: int = 0, task: str = "LOGISTIC_REGRESSION", pool: str = "random",
                             int_ids: bool = False, sizes: str = "uniform", size_alpha: float = 1.3,
                             max_rows: int = 20000):
    """Synthetic GAME data at benchmark scale (vectorised, no per-row Python):

    * ``global`` shard: ``fe_nnz`` Zipf(1.1) features out of ``fe_dim`` + intercept (last column);
    * ``entity`` shard: each entity draws its ``re_nnz`` features per row from a private pool of ``re_dim``
      features of a ``re_vocab`` hashed vocabulary (+ intercept) -> after INDEX_MAP projection every entity has
      ~``re_dim`` coefficients;
    * ``pool="exact"``: instead of random draws, row j of an entity takes pool slots ``[j * re_nnz, (j + 1) *
      re_nnz) mod re_dim`` — every entity then has exactly ``min(re_dim, rows * re_nnz)`` coefficients (e.g. the
      "1k coefficients per entity" GAME config with 20 rows x 50 features);
    * ``sizes="powerlaw"``: rows per entity Pareto(``size_alpha``) distributed (1 .. ``max_rows``, mean
      ``rows_per_entity``) instead of all equal — real GLMix entity sizes: most entities have a few rows (row-space
      solves), a tail has hundreds to thousands (the primal block-diagonal solve, entities with n_e > d_e);
    * id tag ``entityId`` = ``e<global entity index>`` (or the integer index with ``int_ids``; ``entity_offset``
      shifts the range, e.g. per rank);
    * labels from a random ground truth (logistic / linear / Poisson).
    """
    from ..data.game_data import GameData
    rng = np.random.default_rng(seed)
    if sizes == "powerlaw":
        if pool == "exact":
            raise ValueError("pool='exact' needs equal entity sizes")
        u = rng.random(n_entities)
        target = n_entities * rows_per_entity
        xm = float(rows_per_entity) * (size_alpha - 1) / size_alpha
        for _ in range(30):          # scale so that the capped Pareto sizes have the requested mean
            cnt = np.minimum(np.ceil(xm * u ** (-1.0 / size_alpha)), max_rows).astype(np.int64)
            tot = int(cnt.sum())
            if abs(tot - target) <= 0.001 * target:
                break
            xm *= target / tot
        ent = rng.permutation(np.repeat(np.arange(n_entities, dtype=np.int64), cnt))
    elif sizes == "uniform":
        ent = rng.permutation(np.repeat(np.arange(n_entities, dtype=np.int64), rows_per_entity))
    else:
        raise ValueError(f"unknown entity size law {sizes!r}")
    n = len(ent)
    # fixed effect shard
    ranks = np.arange(1, fe_dim)
    p = ranks ** -1.1
    cdf = np.cumsum(p) / p.sum()
    fcol = np.minimum(np.searchsorted(cdf, rng.random((n, fe_nnz))), fe_dim - 2)
    fcol = np.sort(fcol, axis=1)
    dup = np.zeros_like(fcol, dtype=bool)
    dup[:, 1:] = fcol[:, 1:] == fcol[:, :-1]
    fval = np.where(dup, 0.0, rng.random((n, fe_nnz)) + 0.5)
    fcols = np.concatenate([fcol, np.full((n, 1), fe_dim - 1)], 1)
    fvals = np.concatenate([fval, np.ones((n, 1))], 1)
    xg = sp.csr_matrix((fvals.ravel(), fcols.ravel(), np.arange(0, n * (fe_nnz + 1) + 1, fe_nnz + 1)),
                       shape=(n, fe_dim))
    xg.eliminate_zeros()
    # random effect shard: pool slot k of entity e -> feature (hash(e) + k * stride) % re_vocab
    if pool == "exact":
        if re_nnz > re_dim:
            raise ValueError("pool='exact' needs re_nnz <= re_dim")
        srt = np.argsort(ent, kind="stable")
        within = np.empty(n, dtype=np.int64)
        within[srt] = np.arange(n) - np.repeat(np.arange(n_entities) * rows_per_entity, rows_per_entity)
        slot = (within[:, None] * re_nnz + np.arange(re_nnz)[None, :]) % re_dim
        del srt, within
        slot.sort(axis=1)
        rdup = None
    else:
        slot = rng.integers(0, re_dim, size=(n, re_nnz))
        slot = np.sort(slot, axis=1)
        rdup = np.zeros_like(slot, dtype=bool)
        rdup[:, 1:] = slot[:, 1:] == slot[:, :-1]
    gid = ent + entity_offset
    base = (gid * 2654435761) % (re_vocab - 1)
    rcol = (base[:, None] + slot * 40503) % (re_vocab - 1)
    rval = rng.normal(size=(n, re_nnz)) if rdup is None else np.where(rdup, 0.0, rng.normal(size=(n, re_nnz)))
    rc = np.empty((n, re_nnz + 1), dtype=np.int32)
    rc[:, :re_nnz] = rcol
    rc[:, re_nnz] = re_vocab - 1
    del rcol
    rv = np.empty((n, re_nnz + 1))
    rv[:, :re_nnz] = rval
    rv[:, re_nnz] = 1.0
    xr = sp.csr_matrix((rv.ravel(), rc.ravel(), np.arange(0, n * (re_nnz + 1) + 1, re_nnz + 1, dtype=np.int64)),
                       shape=(n, re_vocab))
    del rc, rv
    if rdup is not None:
        xr.sum_duplicates()
        xr.eliminate_zeros()
    # ground truth
    wg = rng.normal(size=fe_dim) * 0.2
    wg[-1] = -0.5
    w_slot = np.random.default_rng(seed + 1).normal(size=re_dim) * 0.5
    zr = (rval * w_slot[slot] if rdup is None else np.where(rdup, 0.0, rval * w_slot[slot])).sum(1) + 0.3 * np.sin(gid)
    del rval, slot
    z = np.asarray(xg @ wg).ravel() + zr
    task = TaskType.parse(task)
    if task == TaskType.LOGISTIC_REGRESSION:
        y = (rng.random(n) < 1.0 / (1.0 + np.exp(-z))).astype(np.float64)
    elif task == TaskType.POISSON_REGRESSION:
        y = rng.poisson(np.exp(np.clip(z * 0.3, -10, 3))).astype(np.float64)
    else:
        y = z + 0.1 * rng.normal(size=n)
    ids = gid.copy() if int_ids else np.char.add("e", gid.astype(str)).astype(object)
    return GameData(y, {"global": xg, "entity": xr}, {"entityId": ids})
