"""GAME coordinates: fixed effect (one GLM over a row-sharded feature shard) and random effect (one GLM per
entity, batched).

Reference: ``photon-lib/.../algorithm/Coordinate.scala:27-80`` (score / initializeModel / updateModel(model,
partialScore) = add the partial score to the offsets, then optimise), ``photon-api/.../algorithm/
FixedEffectCoordinate.scala:35-166``, ``RandomEffectCoordinate.scala:39-222`` and
``RandomEffectCoordinateInProjectedSpace.scala``.

Scores are N-length fp64 tensors aligned with the samples of the training ``GameData`` (no joins). The fixed
effect coordinate keeps ONE device-resident shard for its whole life and only rewrites its offset / weight
vectors per update; the random-effect coordinate keeps its buckets resident and gathers the per-slot offsets
from the partial-score vector (C11 routing) before each batched solve.
"""
from __future__ import annotations

import logging
import os
import time
from typing import Optional

import numpy as np
import torch

from ..constants import EPSILON, TaskType
from ..utils.timing import Timed, phase
from ..data.game_data import GameData
from ..data.matrix import DeviceCSR
from ..data.random_effect import FixedEffectDataConfiguration, RandomEffectDataConfiguration, RandomEffectDataset
from ..function.losses import loss_for_task
from ..models.game import FixedEffectModel, RandomEffectModel
from ..models.glm import Coefficients, model_for_task
from ..normalization.context import NormalizationContext
from ..ops.backend import default_device, make_glm_data
from ..optimization.batched import BatchedGLMData, BatchedResult, batched_lbfgs, batched_tron
from ..optimization.config import GLMOptimizationConfiguration, OptimizerType, RegularizationType
from ..optimization.problem import GLMOptimizationProblem
from ..parallel.dist import DistributedGLMData, is_dist
from ..sampling.samplers import down_sampler_for_task


log = logging.getLogger(__name__)
# data-only solver setup (FE launch tables, RE solver components) at coordinate construction (PML_EAGER_SETUP=0:
# lazily in the first update, as before round 6)
EAGER_SETUP = os.environ.get("PML_EAGER_SETUP", "1") != "0"


def _sync(t):
    """Device sync for phase timing (``PML_SYNC_TIMING=1`` only; asynchronous otherwise)."""
    if os.environ.get("PML_SYNC_TIMING") == "1" and t is not None and t.is_cuda:
        torch.cuda.synchronize(t.device)


def random_effect_tracker_stats(iters: torch.Tensor, reasons: torch.Tensor, seconds: float) -> dict:
    """RandomEffectOptimizationTracker (photon-api/.../RandomEffectOptimizationTracker.scala:100-150): counts of
    convergence reasons and iteration statistics over the entities of one update. Reduced where the tensors live
    (the device): one small transfer of scalars instead of the per-entity arrays."""
    from ..optimization.batched import REASON_CODES
    it = iters.detach().to(torch.float64)
    rc = reasons.detach().to(torch.int64)
    n = it.numel()
    if n == 0:
        return {"entities": 0, "mean_iterations": 0.0, "std_iterations": 0.0, "max_iterations": 0,
                "min_iterations": 0, "convergence_reasons": {}, "seconds": seconds}
    codes = sorted(REASON_CODES)
    hist = torch.stack([(rc == c).sum() for c in codes]).to(torch.float64)
    vals = torch.cat([torch.stack([it.mean(), it.std() if n > 1 else torch.zeros((), dtype=torch.float64,
                                                                                 device=it.device),
                                   it.max(), it.min()]), hist]).cpu().tolist()
    counts = {}
    for code, cnt in zip(codes, vals[4:]):
        if cnt:
            reason = REASON_CODES[code]
            counts["not converged" if reason is None else reason.value] = int(cnt)
    return {"entities": int(n), "mean_iterations": float(vals[0]), "std_iterations": float(vals[1]),
            "max_iterations": int(vals[2]), "min_iterations": int(vals[3]), "convergence_reasons": counts,
            "seconds": seconds}


class Coordinate:
    coordinate_id: str

    def initialize_model(self):
        raise NotImplementedError

    def update_model(self, model, partial_score: Optional[torch.Tensor] = None):
        raise NotImplementedError

    def score(self, model) -> torch.Tensor:
        raise NotImplementedError

    def regularization_term_value(self, model) -> float:
        raise NotImplementedError


class FixedEffectCoordinate(Coordinate):
    def __init__(self, coordinate_id: str, data: GameData, data_config: FixedEffectDataConfiguration,
                 opt_config: GLMOptimizationConfiguration, task, normalization: Optional[NormalizationContext] = None,
                 compute_variance: bool = False, device=None, precision: str = "f64", local_rows=None):
        self.coordinate_id = coordinate_id
        self.data = data
        self.shard_id = data_config.feature_shard_id
        self.task = TaskType.parse(task)
        self.device = torch.device(device) if device is not None else default_device()
        with phase(f"FE {coordinate_id} build: shard view"):
            labeled = data.labeled(self.shard_id)
            if local_rows is not None:  # row sharding for multi-GPU data parallelism
                labeled = labeled.subset(local_rows)
            self.local_rows = local_rows
            self.base_offsets = labeled.offsets.copy()
            self.base_weights = labeled.weights.copy()
            self.labels = labeled.y
        with phase(f"FE {coordinate_id} build: device layout"):
            self.glm_data = make_glm_data(labeled, self.device, precision)
        gd = self.glm_data
        x = data.shards.get(self.shard_id)
        if (isinstance(x, DeviceCSR) and x.data.is_cuda and hasattr(gd, "_build_multi")
                and os.environ.get("PML_FE_OFFLOAD_SHARD", "1") != "0"):
            # rows placed / routed to this rank arrive as a device CSR; the tiled layout now holds them, so the CSR
            # goes to host memory instead of doubling the shard's HBM footprint for the whole fit
            x.offload_to_host()
        if EAGER_SETUP and hasattr(gd, "_build_multi"):
            # every pass of every update uses the shard-wide launch tables: build them with the layout (one-time data
            # setup), not inside the first update
            with phase(f"FE {coordinate_id} build: launch tables"):
                if getattr(gd, "_multi", "unset") == "unset":
                    gd._build_multi()
                if getattr(gd, "_multi_t", "unset") == "unset":
                    gd._build_multi_t()
            if hasattr(gd, "frob_sq"):
                # ||X||_F^2 (the zero point's gradient bound of every update) depends on the data only: computed with
                # the layout, not in the first update (it was ~100 small launches of the cold first sweep)
                with phase(f"FE {coordinate_id} build: Frobenius norm"):
                    gd.frob_sq()
        self.compute_variance = compute_variance
        self.normalization = normalization
        self.set_config(opt_config)
        self.last_tracker = None

    def set_config(self, opt_config: GLMOptimizationConfiguration):
        self.opt_config = opt_config
        self.problem = GLMOptimizationProblem(opt_config, self.task, self.normalization, self.compute_variance)
        rate = opt_config.down_sampling_rate
        self.sampler = down_sampler_for_task(self.task, rate) if rate < 1.0 else None

    @property
    def dim(self) -> int:
        return self.glm_data.dim

    def _data_view(self, data=None):
        data = self.glm_data if data is None else data
        return DistributedGLMData(data) if is_dist() else data

    def initialize_model(self):
        return FixedEffectModel(model_for_task(self.task, Coefficients.zeros(self.dim)), self.shard_id)

    def _device_row_data(self):
        """Base offsets / weights (and the DP row subset) kept on the data's device: the per-update residual
        offsets are formed there (C15: no N-length host round trip per coordinate update)."""
        if getattr(self, "_base_off_t", None) is None:
            dev = getattr(self.glm_data, "device", torch.device("cpu"))
            self._base_off_t = torch.from_numpy(self.base_offsets).to(dev)
            self._rows_t = None if self.local_rows is None else torch.from_numpy(
                np.asarray(self.local_rows, dtype=np.int64)).to(dev)
        return self._base_off_t, self._rows_t

    def update_model(self, model: FixedEffectModel, partial_score: Optional[torch.Tensor] = None):
        base, rows = self._device_row_data()
        off = base
        fused = False
        if partial_score is not None:
            ps = partial_score.detach().to(base.device, torch.float64)
            ps = ps if rows is None else ps[rows]
            fn = getattr(self.glm_data, "set_offsets_sum", None)
            fused = fn is not None and fn(base, ps)          # sum + cast + margin shift in one pass
            if not fused:
                off = base + ps
        if not fused:
            self.glm_data.set_offsets(off)
        gd = self.glm_data
        if self.sampler is not None:
            self._apply_down_sampling()
            gd = self._sampled_shard() or gd
        n0 = (getattr(gd, "n_fwd", 0), getattr(gd, "n_t", 0))
        glm = self.problem.run(self._data_view(gd), model.glm if model is not None else None, dim=self.dim)
        self.last_tracker = self.problem.tracker
        if log.isEnabledFor(logging.DEBUG) and hasattr(gd, "n_passes"):
            log.debug("FE %s: %d forward + %d transpose passes in the update (%s iterations)", self.coordinate_id,
                      getattr(gd, "n_fwd", 0) - n0[0], getattr(gd, "n_t", 0) - n0[1],
                      getattr(self.last_tracker, "iterations", "?"))
        # restore full weights for scoring/evaluation
        if self.sampler is not None:
            self._restore_weights()
        # the coefficients stay where the optimizer left them (the device): scoring reads the cached margins of
        # this very tensor, the next update warm-starts from it without an 8-byte-per-feature host round trip and
        # without a device comparison to re-identify it; writers / diagnostics copy to the host themselves
        return FixedEffectModel(glm.update_coefficients(
            Coefficients(glm.coefficients.means.detach(), None if glm.coefficients.variances is None
                         else glm.coefficients.variances.detach())), self.shard_id)

    def _row_ids(self) -> np.ndarray:
        """Global row ids of this coordinate's rows (the down-sampling hash input: rank-independent samples)."""
        return np.arange(len(self.labels)) if self.local_rows is None else np.asarray(self.local_rows)

    def _apply_down_sampling(self):
        """K20: rewrite the device weight vector in place (downsample_kernel) — no host arrays, no upload per
        update; host data backends get the same weights from the host twin of the hash."""
        gd = self.glm_data
        wt = getattr(gd, "wt", None)
        if isinstance(wt, torch.Tensor) and wt.is_cuda:
            if getattr(self, "_w_base_dev", None) is None:
                self._w_base_dev = wt.clone()
                self._rowid_dev = torch.from_numpy(self._row_ids().astype(np.int64)).to(wt.device)
            self.sampler.sample_weights_device(gd.y, self._w_base_dev, self._rowid_dev, out=wt)
            gd.mark_weights_changed()
            return
        wts = self.sampler.sample_weights(self.labels, self.base_weights, self._row_ids())
        gd.set_weights(torch.from_numpy(np.asarray(wts, dtype=np.float64)))

    def _sampled_shard(self):
        """K20 work saving on the device path: the update runs on a copy of the shard that holds only the kept
        rows' entries (``DeviceGLMData.row_sampled``), so at rate r each pass streams ~r of the data, as the
        reference's physically down-sampled RDD does. ``PML_DS_COMPACT=0`` keeps the zero-weight full passes."""
        gd = self.glm_data
        wt = getattr(gd, "wt", None)
        if (os.environ.get("PML_DS_COMPACT", "1") == "0" or not hasattr(gd, "row_sampled")
                or not isinstance(wt, torch.Tensor) or not wt.is_cuda):
            return None
        return gd.row_sampled(wt[: gd.n_rows] > 0)

    def _restore_weights(self):
        wt = getattr(self.glm_data, "wt", None)
        if isinstance(wt, torch.Tensor) and wt.is_cuda and getattr(self, "_w_base_dev", None) is not None:
            wt.copy_(self._w_base_dev)
            self.glm_data.mark_weights_changed()
        else:
            self.glm_data.set_weights(torch.from_numpy(self.base_weights))

    def score(self, model: FixedEffectModel) -> torch.Tensor:
        if self.local_rows is None:
            w = model.glm.coefficients.means.to(self.glm_data.device, torch.float64)
            return self.glm_data.margins(w).to(self.device, torch.float64)
        return model.score(self.data, self.device)

    def regularization_term_value(self, model: FixedEffectModel) -> float:
        return self.problem.regularization_term_value(model.glm)


_RS_WARM = object()   # warm-start marker: the last segmented solve kept only row-space coordinates


class RandomEffectCoordinate(Coordinate):
    """Per-entity GLMs solved in size buckets on the device (K7)."""

    def __init__(self, coordinate_id: str, data: GameData, data_config: RandomEffectDataConfiguration,
                 opt_config: GLMOptimizationConfiguration, task, compute_variance: bool = False, device=None,
                 dtype=torch.float64, entity_subset=None, layout: str = "auto"):
        self.coordinate_id = coordinate_id
        self.data = data
        self.data_config = data_config
        self.task = TaskType.parse(task)
        self.loss = loss_for_task(self.task)
        self.device = torch.device(device) if device is not None else default_device()
        with phase(f"RE {coordinate_id} build: dataset"):
            self.dataset = RandomEffectDataset(data, data_config, self.device, dtype, entity_subset=entity_subset,
                                               layout=layout)
        self.compute_variance = compute_variance
        self.base_offsets = torch.from_numpy(data.offsets).to(self.device)
        self.set_config(opt_config)
        self._W = {}  # projected-space warm-start state per bucket
        self._returned = None  # the model object the last update returned (its solver state is in _W / _rs)
        self.last_stats = {}
        if EAGER_SETUP and self.dataset.layout == "segmented" and self.device.type == "cuda":
            # the solver components (row-space Gram factors, the fused batch's gathered rows, launch classes) depend
            # on the data only: built with the dataset, as the reference builds its RandomEffectDataSet up front
            # (RandomEffectDataSet.scala:239-279), so the first coordinate-descent update is a solve
            cfg = self.opt_config
            reg, lam = cfg.regularization_context, cfg.regularization_weight
            with phase(f"RE {coordinate_id} build: solver components"):
                comps = self._components(reg.l1_weight(lam), cfg.optimizer_config)
                if comps is not None and os.environ.get("PML_RE_OVERLAP", "1") != "0":
                    # the side streams of the concurrent row-space / pass-path solves (creating a prioritised stream
                    # is ~16 ms on first use): made with the components, not inside the first update
                    if comps[0] is not None and comps[1] is not None:
                        self._side_stream = torch.cuda.Stream(
                            self.device, priority=int(os.environ.get("PML_RE_SIDE_PRIORITY", "0")))
                    if comps[2] is not None and comps[1] is not None:
                        self._sub_stream = torch.cuda.Stream(
                            self.device, priority=int(os.environ.get("PML_RE_SUB_PRIORITY", "-1")))

    # The tracker statistics of the last update (random_effect_tracker_stats) are reduced on first read: the masked
    # selection of active entities and the dozen small reductions behind them (a stream synchronisation) stay off
    # the coordinate-descent critical path unless someone looks at them.
    @property
    def last_stats(self) -> dict:
        thunk = self.__dict__.get("_stats_thunk")
        if thunk is not None:
            self.__dict__["_stats"] = thunk()
            self.__dict__["_stats_thunk"] = None
        return self.__dict__.get("_stats", {})

    @last_stats.setter
    def last_stats(self, value: dict):
        self.__dict__["_stats"], self.__dict__["_stats_thunk"] = value, None

    def _defer_stats(self, iters: torch.Tensor, reasons: torch.Tensor, act: torch.Tensor, seconds: float):
        self.__dict__["_stats_thunk"] = lambda: random_effect_tracker_stats(iters[act], reasons[act], seconds)

    def set_config(self, opt_config: GLMOptimizationConfiguration):
        rt = opt_config.regularization_context.regularization_type
        if opt_config.optimizer_config.optimizer_type == OptimizerType.TRON and rt in (
                RegularizationType.L1, RegularizationType.ELASTIC_NET):
            raise ValueError("TRON optimizer incompatible with L1 regularization")
        self.opt_config = opt_config
        self._reset_warm_state()

    def _reset_warm_state(self):
        """Forget cached solver state (bucket W, segmented W, row-space beta, lazy primal model)."""
        self._W = {}
        self._returned = None
        if getattr(self, "_rs", None) is not None:
            self._rs.beta = None
        comps = getattr(self, "_comps", None)
        if comps is not None and comps[1] is not None:
            comps[1].W = None
        self._sub_W = None

    def initialize_model(self):
        ds = self.dataset
        return RandomEffectModel(self.data_config.random_effect_type, self.data_config.feature_shard_id, self.task,
                                 ds.entity_ids, ds.dim, np.zeros(0, np.int64), np.zeros(0))

    def _warm_start(self, b, bucket, model: Optional[RandomEffectModel]):
        key = b
        dev, dt = self.device, self.dataset.dtype
        B, _, d = bucket.X.shape
        if key in self._W and self._W[key].shape == (B, d):
            return self._W[key]
        W = torch.zeros(B, d, dtype=dt, device=dev)
        ds = self.dataset
        if model is not None and model.nnz and ds.projector_type.kind.value == "INDEX_MAP":
            # map original-space coefficients into each entity's local index space
            ptr, feat = ds.projection.ptr, ds.projection.feat
            ents = bucket.entities
            b_idx = np.concatenate([np.full(ds.d_local[e], i) for i, e in enumerate(ents)]) if len(ents) else []
            c_idx = np.concatenate([np.arange(ds.d_local[e]) for e in ents]) if len(ents) else []
            gf = np.concatenate([feat[ptr[e]:ptr[e + 1]] for e in ents]) if len(ents) else []
            mi = model.entity_index(ds.entity_ids[np.repeat(ents, ds.d_local[ents])])
            k = mi.astype(np.int64) * model.dim + np.asarray(gf, dtype=np.int64)
            pos = np.searchsorted(model.keys, k)
            pos_c = np.minimum(pos, len(model.keys) - 1)
            hit = (pos < len(model.keys)) & (model.keys[pos_c] == k) & (mi >= 0)
            vals = np.where(hit, model.values[pos_c], 0.0)
            Wn = np.zeros((B, d))
            Wn[np.asarray(b_idx, dtype=np.int64), np.asarray(c_idx, dtype=np.int64)] = vals
            W = torch.from_numpy(Wn).to(dev, dt)
        return W

    def update_model(self, model: Optional[RandomEffectModel], partial_score: Optional[torch.Tensor] = None):
        ds = self.dataset
        cfg = self.opt_config
        reg, lam = cfg.regularization_context, cfg.regularization_weight
        l1, l2 = reg.l1_weight(lam), reg.l2_weight(lam)
        offs = self.base_offsets if partial_score is None else self.base_offsets + partial_score.to(self.device)
        if model is None or model is not self._returned:
            # the cached solver state belongs to the model this coordinate returned last; any other starting model
            # (a fresh start, another configuration's best model) is mapped from its coefficients instead
            self._reset_warm_state()
        out = (self._update_segmented(model, offs, l1, l2) if ds.layout == "segmented"
               else self._update_buckets(model, offs, l1, l2))
        self._returned = out
        return out

    def _update_buckets(self, model, offs, l1: float, l2: float):
        ds, cfg = self.dataset, self.opt_config
        keys, vals, vars_ = [], [], []
        iters, reasons = [], []
        t_start = time.time()
        for b, bucket in enumerate(ds.buckets):
            O = ds.bucket_offsets(bucket, offs)
            bd = BatchedGLMData(bucket.X, bucket.y, O, bucket.w)
            W0 = self._warm_start(b, bucket, model)
            oc = cfg.optimizer_config
            fz = self._dense_fused(b, bucket, l1)
            if fz is not None:
                r = fz.solve(self.loss, l2, W0, O, oc.tolerance, oc.maximum_iterations)
                res = BatchedResult(r.W.to(W0.dtype), r.f, r.iters, r.reason)
            elif oc.optimizer_type == OptimizerType.TRON:
                res = batched_tron(bd, self.loss, l2, W0, oc.tolerance, oc.maximum_iterations)
            else:
                res = batched_lbfgs(bd, self.loss, l2, W0, oc.tolerance, oc.maximum_iterations, l1=l1)
            self._W[b] = res.W
            iters.append(res.iters)
            reasons.append(res.reason)
            W = res.W
            var = None
            if self.compute_variance and self.loss.twice_differentiable:
                var = 1.0 / (bd.hdiag(self.loss, W, l2) + EPSILON)
            k, v, vv = self._to_original(bucket, W, var)
            keys.append(k)
            vals.append(v)
            if vv is not None:
                vars_.append(vv)
        it = torch.cat([i.cpu() for i in iters]) if iters else torch.zeros(0)
        rs = torch.cat([r.cpu() for r in reasons]) if reasons else torch.zeros(0, dtype=torch.long)
        self.last_stats = random_effect_tracker_stats(it, rs, time.time() - t_start)
        keys = np.concatenate(keys) if keys else np.zeros(0, np.int64)
        vals = np.concatenate(vals) if vals else np.zeros(0)
        variances = np.concatenate(vars_) if vars_ else None
        return RandomEffectModel(self.data_config.random_effect_type, self.data_config.feature_shard_id, self.task,
                                 ds.entity_ids, ds.dim, keys, vals, variances)

    def _dense_fused(self, b: int, bucket, l1: float):
        """The fused per-entity TRON of a dense bucket (``entity_tron.DenseEntityTronBatch``, built once per
        bucket), or None when it does not apply (L-BFGS / OWL-QN, L1, constraints, CPU, non-smooth loss, d > 2048)."""
        from ..optimization.entity_tron import FUSED_DMAX, DenseEntityTronBatch, fused_eligible
        oc = self.opt_config.optimizer_config
        opt = "TRON" if oc.optimizer_type == OptimizerType.TRON else "LBFGS"
        if (not fused_eligible(self.loss, opt, l1, oc.constraint_map, bucket.X.device)
                or bucket.X.shape[2] > FUSED_DMAX or bucket.X.numel() == 0):
            return None
        cache = self.__dict__.setdefault("_dense_fz", {})
        if b not in cache:
            cache[b] = DenseEntityTronBatch(bucket.X, bucket.y, bucket.w)
        return cache[b]

    def _update_segmented(self, model, offs, l1: float, l2: float):
        """All entities as one block-diagonal problem (``SegmentedGLMData``). With the fused primal TRON
        available (``optimization/entity_tron.py``) the entities are split into components — row-space batch,
        fused per-entity TRON, leftover pass-path subset — each keeping its own solver state
        (:meth:`_update_components`); otherwise one TRON / L-BFGS over the concatenated per-entity coefficient
        vector with the row-space batch frozen."""
        ds, cfg = self.dataset, self.opt_config
        seg = ds.seg
        offs = offs.to(seg.y.device, torch.float64)
        seg.o = offs if getattr(ds, "seg_rows_identity", False) else offs[ds.seg_rows]
        seg._dzz_key = None
        comps = self._components(l1, cfg.optimizer_config)
        if comps is not None:
            return self._update_components(comps, model, l1, l2)
        # previous update kept only beta (lazy primal model): the row-space solve warm-starts from it directly
        prev_lazy = self._W.get("seg") is _RS_WARM
        W0 = None if prev_lazy else self._warm_start_segmented(model)
        t_start = time.time()
        oc = cfg.optimizer_config
        with Timed(f"RE {self.coordinate_id}: row-space setup", log, logging.DEBUG):
            rs = self._row_space(l1, oc)
        frozen = None
        if rs is not None and rs.B:
            # wide entities (n_e <= d_e) solved exactly in their row space (optimization/row_space.py)
            opt = "TRON" if oc.optimizer_type == OptimizerType.TRON else "LBFGS"
            with Timed(f"RE {self.coordinate_id}: row-space solve", log, logging.DEBUG):
                rres = rs.solve(self.loss, l2, opt, W0, oc.tolerance, oc.maximum_iterations,
                                reuse_beta=self._W.get("seg") is not None)
                _sync(rres.W)
            frozen = rs.mask
            n_e = seg.row_ptr[1:] - seg.row_ptr[:-1]
            all_rs = bool((frozen | (n_e == 0)).all())   # nothing left for the primal path
            if not all_rs:
                if W0 is None:
                    W0 = self._lazy_W()
                W0 = torch.where(seg.bexp(frozen), torch.zeros_like(W0), W0)
        if frozen is None or not all_rs:
            if W0 is None:
                W0 = self._lazy_W()
            with Timed(f"RE {self.coordinate_id}: primal block-diagonal solve", log, logging.DEBUG):
                sub = self._primal_subset(frozen) if frozen is not None else None
                if sub is not None:
                    # only the entities NOT solved in their row space, on their own rows / coefficients
                    sub.seg.o = seg.o[sub.rows]
                    sub.seg._dzz_key = None
                    prob, W0p = sub.seg, W0[sub.cols].contiguous()
                    fz = None
                else:
                    prob, W0p, fz = seg, W0, frozen
                if oc.optimizer_type == OptimizerType.TRON:
                    res = batched_tron(prob, self.loss, l2, W0p, oc.tolerance, oc.maximum_iterations, frozen=fz)
                else:
                    res = batched_lbfgs(prob, self.loss, l2, W0p, oc.tolerance, oc.maximum_iterations, l1=l1,
                                        frozen=fz)
                if sub is not None:
                    W_all = torch.zeros_like(W0).index_copy_(0, sub.cols, res.W)
                    iters = torch.zeros(seg.B, dtype=torch.long, device=W0.device).index_copy_(0, sub.entities,
                                                                                             res.iters)
                    reasons = torch.zeros(seg.B, dtype=torch.long, device=W0.device).index_copy_(0, sub.entities,
                                                                                               res.reason)
                else:
                    W_all, iters, reasons = res.W, res.iters, res.reason
        else:
            W_all = None
            iters = torch.zeros(seg.B, dtype=torch.long, device=seg.y.device)
            reasons = torch.zeros(seg.B, dtype=torch.long, device=seg.y.device)
        self._rs_scores = None
        need_var = self.compute_variance and self.loss.twice_differentiable
        if (frozen is not None and all_rs and not need_var and not len(self.dataset.passive_rows)
                and os.environ.get("PML_RE_LAZY_PRIMAL", "1") != "0"):
            # every entity solved in its row space: scores are L beta, ||w||^2 = ||beta||^2, and the primal
            # coefficients w = X^T L^-T beta (one transpose pass over the block-diagonal data) are produced only
            # when the model is read
            beta = rres.W
            self._rs_scores = rs.margins(beta)
            self._lazy_W = lambda: rs.to_primal(beta)
            self._W["seg"] = _RS_WARM
            n_iter = torch.zeros(seg.B, dtype=torch.long, device=beta.device).index_copy(0, rs.ents, rres.iters)
            n_reason = torch.zeros(seg.B, dtype=torch.long, device=beta.device).index_copy(0, rs.ents, rres.reason)
            act = self._active_mask(n_iter.device)
            self._defer_stats(n_iter, n_reason, act, time.time() - t_start)
            sum_sq = float(torch.linalg.vector_norm(torch.where(rs.valid, beta, torch.zeros_like(beta)))) ** 2
            out = RandomEffectModel(self.data_config.random_effect_type, self.data_config.feature_shard_id, self.task,
                                    ds.entity_ids, ds.dim, ds.projection_keys_t, self._lazy_W, None, sum_sq=sum_sq)
            self._last = (out, None)
            return out
        if frozen is not None:
            with Timed(f"RE {self.coordinate_id}: row-space -> primal", log, logging.DEBUG):
                Wp = rs.to_primal(rres.W)
                W_all = Wp if W_all is None else W_all + Wp
                _sync(W_all)
            if all_rs:  # active-row scores X w = L beta without a pass over the sparse data
                self._rs_scores = rs.margins(rres.W)
            iters = iters.index_copy(0, rs.ents, rres.iters)
            reasons = reasons.index_copy(0, rs.ents, rres.reason)
        res = BatchedResult(W_all, None, iters, reasons)
        self._W["seg"] = res.W
        act = self._active_mask(res.iters.device)
        self._defer_stats(res.iters, res.reason, act, time.time() - t_start)
        W = res.W.detach()
        var = None
        if self.compute_variance and self.loss.twice_differentiable:
            var = 1.0 / (seg.hdiag(self.loss, res.W, l2) + EPSILON)
        # the model keeps the projected keys (entity * dim + feature, sorted, aligned with W) without compaction:
        # W is dense in the projected space, and zeros are harmless (dropped at save, <1e-4 as in the reference);
        # compacting 1.25e9 coefficients per update was ~40 GB of traffic at config 5
        out = RandomEffectModel(self.data_config.random_effect_type, self.data_config.feature_shard_id, self.task,
                                ds.entity_ids, ds.dim, ds.projection_keys_t, W, var)
        self._last = (out, res.W)
        return out

    def _components(self, l1: float, oc):
        """Solver components of the segmented coordinate, built once per dataset: ``(rs, fused, sub)`` = the
        row-space batch (wide entities, ``row_space.py``), the fused per-entity primal TRON batch
        (``entity_tron.py``) and the leftover entities as a block-diagonal sub-problem for the pass path (any of
        them None when empty). None when the fused primal TRON does not apply to this configuration or the
        segmented CSR was already released by an earlier split."""
        from ..optimization.entity_tron import EntityTronBatch, fused_eligible
        opt = "TRON" if oc.optimizer_type == OptimizerType.TRON else "LBFGS"
        ds = self.dataset
        seg = ds.seg
        if not fused_eligible(self.loss, opt, l1, oc.constraint_map, seg.y.device):
            return None
        cached = getattr(self, "_comps", None)
        if cached is not None:
            return cached
        if getattr(ds, "_seg_csr", None) is None:
            return None
        with Timed(f"RE {self.coordinate_id}: solver components", log, logging.DEBUG):
            with Timed(f"RE {self.coordinate_id}: row-space batch", log, logging.DEBUG):
                rs = self._row_space(l1, oc)
                rs = rs if rs is not None and rs.B else None
            n_e = seg.row_ptr[1:] - seg.row_ptr[:-1]
            done = rs.mask.clone() if rs is not None else torch.zeros(seg.B, dtype=torch.bool, device=seg.y.device)
            with Timed(f"RE {self.coordinate_id}: fused primal batch", log, logging.DEBUG):
                fused = EntityTronBatch(ds, (~done) & (n_e > 0))
            if fused.B:
                done |= fused.mask
            else:
                fused = None
            rest = (~done) & (n_e > 0)
            sub = ds.entity_subset(rest) if bool(rest.any()) else None
            ds.release_csr()
            # do the three components' coefficient ranges cover the whole packed vector? Then the model's primal
            # vector needs no zero fill before they write it (each component writes whole entity ranges)
            cov = 0 if rs is None else int((seg.col_ptr[rs.ents + 1] - seg.col_ptr[rs.ents]).sum())
            cov += (0 if fused is None else int(fused.cols.numel())) + (0 if sub is None else int(sub.cols.numel()))
            self._w_covered = cov == int(seg.col_ptr[-1])
        self._comps = (rs, fused, sub)
        self._sub_W = None
        log.debug("RE %s: %d row-space, %d fused primal, %d pass-path entities", self.coordinate_id,
                  0 if rs is None else rs.B, 0 if fused is None else fused.B,
                  0 if sub is None else sub.entities.numel())
        return self._comps

    def solver_routing(self) -> dict:
        """Where this coordinate's entities are solved (after its first update): row-space / fused primal /
        pass-path counts, the fused batch's register-resident clusters and launches. Diagnostics for benchmarks."""
        comps = getattr(self, "_comps", None)
        if comps is None:
            return {}
        rs, fused, sub = comps
        out = {"row_space": 0 if rs is None else int(rs.B), "fused": 0 if fused is None else int(fused.B),
               "pass_path": 0 if sub is None else int(sub.entities.numel())}
        if fused is not None:
            out["fused_launches"] = len(fused.launches)
            out["heavy_to_pass_path"] = int(fused.n_heavy)
            out["quad_rows"] = bool(fused.quad)
            r = fused.res
            if r is not None:
                k = r["t0"][1:] - r["t0"][:-1]
                out["resident"] = {"entities": r["n"], "clusters": r["clusters"], "workgroups": r["tickets"],
                                   "largest_cluster": int(k.max()), "clusters_ge8": int((k >= 8).sum()),
                                   "error_flag_checks": int(getattr(self, "_res_checks", 0))}
        return out

    def _update_components(self, comps, model, l1: float, l2: float):
        """One update over the solver components (see :meth:`_components`). Each component warm-starts from its
        own last solution (the row-space beta, the fused batch's packed W, the subset's W) unless the starting
        model is not the one this coordinate returned last — then from that model's coefficients. Scores come
        out of the solves (row space: L beta; fused: the kernel's margins; pass path: one forward pass over the
        subset only), and the primal coefficient vector is assembled only when the model is read."""
        from ..optimization.batched import batched_tron
        rs, fused, sub = comps
        ds, oc = self.dataset, self.opt_config.optimizer_config
        seg = ds.seg
        dev = seg.y.device
        warm = self._W.get("seg")
        foreign = warm is not _RS_WARM and model is not None and model.nnz > 0
        W0 = self._warm_start_segmented(model) if foreign else None
        t_start = time.time()
        iters = torch.zeros(seg.B, dtype=torch.long, device=dev)
        reasons = torch.zeros_like(iters)
        z = torch.zeros(seg.y.numel(), dtype=torch.float64, device=dev)     # x.w per row (segmented order)
        sum_sq = torch.zeros((), dtype=torch.float64, device=dev)
        parts = {}

        def run_rs(prep=None):
            with Timed(f"RE {self.coordinate_id}: row-space solve", log, logging.DEBUG):
                rres = rs.solve(self.loss, l2, "TRON", W0, oc.tolerance, oc.maximum_iterations,
                                reuse_beta=not foreign, prep=prep)
                _sync(rres.W)
            # the handled rows' margins go straight into the update's per-row vector (the fused / pass-path rows
            # are disjoint), not into a zero vector added afterwards
            return (rres, rs.margins(rres.W, out=z),
                    torch.where(rs.valid, rres.W, torch.zeros_like(rres.W)).square().sum())

        # the row-space and fused solves touch disjoint entities: with both present the row-space kernels run on a
        # side stream, concurrently with the fused launch (they fill its tail and its host-side gaps)
        overlap = (rs is not None and fused is not None and dev.type == "cuda"
                   and os.environ.get("PML_RE_OVERLAP", "1") != "0")
        rs_out = None
        if rs is not None and not overlap:
            rs_out = run_rs()
        main = side = None
        rs_prep = None
        if overlap:
            # the row-space solve's input passes (warm-start copy, per-slot offsets) run here, on the idle device,
            # before the fused launch takes every CU
            rs_prep = rs.prepare(W0, reuse_beta=not foreign)
            main = torch.cuda.current_stream(dev)
            if getattr(self, "_side_stream", None) is None:
                self._side_stream = torch.cuda.Stream(dev, priority=int(os.environ.get("PML_RE_SIDE_PRIORITY", "0")))
            side = self._side_stream
            side.wait_stream(main)                 # offsets / warm starts written on the main stream
            for t in rs_prep:
                t.record_stream(side)              # allocated on the main stream, read on the side stream
        # the pass-path entities (e.g. a heavy tail too long for the fused kernels) likewise run on their own
        # stream next to the fused launch: their passes are grid-wide and their host-side control only waits on
        # that stream
        sub_async = (sub is not None and fused is not None and dev.type == "cuda"
                     and os.environ.get("PML_RE_OVERLAP", "1") != "0")
        sub_stream = None
        sub_in = None
        if sub_async:
            main = torch.cuda.current_stream(dev)
            if getattr(self, "_sub_stream", None) is None:
                # the pass path is a long chain of short launches next to the saturating fused launch: a
                # high-priority stream lets its workgroups take CUs first as they free up (PML_RE_SUB_PRIORITY;
                # game5heavy RE 62.4 -> 61.0 ms; the row-space side stream measured no better at high priority,
                # scripts/gpu_r5_prio.sh)
                self._sub_stream = torch.cuda.Stream(dev, priority=int(os.environ.get("PML_RE_SUB_PRIORITY", "-1")))
            sub_stream = self._sub_stream
            sub_in = self._sub_inputs(sub, seg, W0)          # on the main stream, before the fused launch
            sub_stream.wait_stream(main)
            sub_in.record_stream(sub_stream)
        fres = None
        if fused is not None:
            with Timed(f"RE {self.coordinate_id}: fused primal solve", log, logging.DEBUG):
                fres = fused.solve(self.loss, l2, None if W0 is None else W0[fused.cols], seg.o[fused.rows],
                                   oc.tolerance, oc.maximum_iterations)
                _sync(fres.W)
            iters.index_copy_(0, fused.ents, fres.iters)
            reasons.index_copy_(0, fused.ents, fres.reason)
            if overlap:
                with torch.cuda.stream(side):
                    rs_out = run_rs(rs_prep)
                for t in (rs_out[0].W, rs_out[0].iters, rs_out[0].reason, rs_out[1], rs_out[2]):
                    t.record_stream(main)
            z.index_copy_(0, fused.rows, fres.z)
            sum_sq += fres.W.square().sum()
            parts["fused"] = fres.W
        if sub is not None:
            with Timed(f"RE {self.coordinate_id}: primal block-diagonal solve", log, logging.DEBUG):
                if sub_async:
                    with torch.cuda.stream(sub_stream):
                        res, z_sub = self._solve_sub(sub, sub_in, l2, oc)
                    main.wait_stream(sub_stream)
                    for t in (res.W, res.iters, res.reason, z_sub):
                        t.record_stream(main)
                else:
                    res, z_sub = self._solve_sub(sub, self._sub_inputs(sub, seg, W0), l2, oc)
                _sync(res.W)
            self._sub_W = res.W
            iters.index_copy_(0, sub.entities, res.iters)
            reasons.index_copy_(0, sub.entities, res.reason)
            z.index_copy_(0, sub.rows, z_sub)
            sum_sq += res.W.square().sum()
            parts["sub"] = res.W
        if fres is not None and rs_out is None:
            fres.check_error()
            self._res_checks = getattr(self, "_res_checks", 0) + (fres.err is not None)
        if rs_out is not None:
            if overlap:
                main.wait_stream(side)
            rres, z_rs, ss_rs = rs_out
            if fres is not None:
                fres.check_error()                 # after the side-stream launch was queued
                self._res_checks = getattr(self, "_res_checks", 0) + (fres.err is not None)
            iters.index_copy_(0, rs.ents, rres.iters)
            reasons.index_copy_(0, rs.ents, rres.reason)
            if z_rs is not z:
                z += z_rs
            sum_sq += ss_rs
            parts["rs"] = rres.W
        del W0

        def primal(parts=parts):
            """The primal coefficient vector over all entities (projected keys order)."""
            W = rs.to_primal(parts["rs"], fill=not getattr(self, "_w_covered", False)) if "rs" in parts else \
                torch.zeros(ds.d_total, dtype=torch.float64, device=dev)
            if "fused" in parts:
                W.index_copy_(0, fused.cols, parts["fused"])
            if "sub" in parts:
                W.index_copy_(0, sub.cols, parts["sub"])
            return W

        self._W["seg"] = _RS_WARM
        self._rs_scores = z
        act = self._active_mask(dev)
        self._defer_stats(iters, reasons, act, time.time() - t_start)
        need_var = self.compute_variance and self.loss.twice_differentiable
        if need_var:
            W = primal()
            var = 1.0 / (seg.hdiag(self.loss, W, l2) + EPSILON)
            out = RandomEffectModel(self.data_config.random_effect_type, self.data_config.feature_shard_id,
                                    self.task, ds.entity_ids, ds.dim, ds.projection_keys_t, W, var)
        else:
            self._lazy_W = primal
            out = RandomEffectModel(self.data_config.random_effect_type, self.data_config.feature_shard_id,
                                    self.task, ds.entity_ids, ds.dim, ds.projection_keys_t, primal, None,
                                    sum_sq=float(sum_sq))
        self._last = (out, None)
        return out

    def _sub_inputs(self, sub, seg, W0) -> torch.Tensor:
        """Warm start of the pass-path subset (its offsets are set on ``sub.seg`` here too)."""
        if W0 is not None:
            W0s = W0[sub.cols].contiguous()
        elif getattr(self, "_sub_W", None) is not None:
            W0s = self._sub_W
        else:
            W0s = torch.zeros(sub.cols.numel(), dtype=torch.float64, device=seg.y.device)
        sub.seg.o = seg.o[sub.rows]
        sub.seg._dzz_key = None
        return W0s

    def _solve_sub(self, sub, W0s, l2: float, oc):
        """Block-diagonal TRON over the pass-path subset (on the current stream); (result, its margins)."""
        from ..optimization.batched import batched_tron
        o = sub.seg.o
        if o.is_cuda:
            o.record_stream(torch.cuda.current_stream(o.device))     # formed on the main stream
        res = batched_tron(sub.seg, self.loss, l2, W0s, oc.tolerance, oc.maximum_iterations)
        return res, sub.seg.glm.matvec(res.W)

    def _active_mask(self, device) -> torch.Tensor:
        """Entities with active data (bool, on ``device``; uploaded once)."""
        m = getattr(self, "_act_mask", None)
        if m is None or m.device != torch.device(device):
            m = torch.from_numpy(self.dataset.n_active > 0).to(device)
            self._act_mask = m
        return m

    def _primal_subset(self, frozen: torch.Tensor):
        """Sub-problem of the entities outside the row-space batch (built once per row-space batch; the kept
        segmented CSR is released afterwards). None when every entity with data is frozen or the data keeps no
        CSR (then the frozen mask is used on the whole problem)."""
        if os.environ.get("PML_RE_PRIMAL_SUBSET", "1") == "0":
            return None
        cached = getattr(self, "_sub", None)
        if cached is not None and cached[0] is frozen:
            return cached[1]
        ds = self.dataset
        if getattr(ds, "_seg_csr", None) is None:
            return None
        seg = ds.seg
        n_e = seg.row_ptr[1:] - seg.row_ptr[:-1]
        mask = (~frozen) & (n_e > 0)
        if not bool(mask.any()):
            return None
        sub = ds.entity_subset(mask)
        ds.release_csr()
        self._sub = (frozen, sub)
        return sub

    def _row_space(self, l1: float, oc):
        """Row-space batch for the wide entities (built once per dataset), or None when not applicable."""
        from ..optimization.row_space import RowSpaceBatch, row_space_eligible
        if os.environ.get("PML_RE_ROW_SPACE", "1") == "0" or not row_space_eligible(l1, oc.constraint_map):
            return None
        if getattr(self, "_rs", None) is None:
            self._rs = RowSpaceBatch(self.dataset.seg, nmax=int(os.environ.get("PML_RS_NMAX", "128")),
                                     csr=getattr(self.dataset, "_seg_csr", None))
        return self._rs

    def _warm_start_segmented(self, model):
        ds = self.dataset
        dev = ds.seg.y.device
        prev = self._W.get("seg")
        if prev is not None and prev.numel() == ds.d_total:
            return prev
        if model is None or model.nnz == 0:
            return torch.zeros(ds.d_total, dtype=torch.float64, device=dev)
        # map (entity, feature) of every projected coefficient to the model's entity numbering, look up on device
        mi = torch.from_numpy(model.entity_index(ds.entity_ids).astype(np.int64)).to(dev)[ds.col_entity_t]
        k = mi * model.dim + ds.projection_keys_t % ds.dim
        mk, mv = model.tensors(dev)
        pos = torch.searchsorted(mk, k).clamp(max=mk.numel() - 1)
        hit = (mk[pos] == k) & (mi >= 0)
        return torch.where(hit, mv[pos], torch.zeros_like(mv[pos]))

    def _to_original(self, bucket, W: torch.Tensor, var: Optional[torch.Tensor]):
        ds = self.dataset
        kind = ds.projector_type.kind.value
        Wn = W.detach().cpu().numpy()
        Vn = None if var is None else var.detach().cpu().numpy()
        ents = bucket.entities
        if kind == "INDEX_MAP":
            ptr, feat = ds.projection.ptr, ds.projection.feat
            dl = ds.d_local[ents]
            b_idx = np.repeat(np.arange(len(ents)), dl)
            c_idx = np.concatenate([np.arange(x) for x in dl]) if len(ents) else np.zeros(0, np.int64)
            gf = np.concatenate([feat[ptr[e]:ptr[e + 1]] for e in ents]) if len(ents) else np.zeros(0, np.int64)
            vals = Wn[b_idx, c_idx]
            keys = np.repeat(ents, dl).astype(np.int64) * ds.dim + gf
            vv = None if Vn is None else Vn[b_idx, c_idx]
        else:
            if kind == "RANDOM" and W.is_cuda:
                # back-projection W P (and V P^2) on the matrix cores: gemm_nt_mfma_kernel, fp64 MFMA
                from ..ops.native import gemm_nt
                PT = ds._matrix_t(W.device)
                orig = gemm_nt(W.detach().to(torch.float64).contiguous(), PT).cpu().numpy()
                vorig = None if var is None else gemm_nt(var.detach().to(torch.float64).contiguous(),
                                                         (PT * PT).contiguous()).cpu().numpy()
            elif kind == "RANDOM":
                orig = Wn @ ds.matrix  # [B, D]
                vorig = None if Vn is None else Vn @ (ds.matrix ** 2)
            else:
                orig, vorig = Wn, Vn
            b_idx, f_idx = np.nonzero(orig)
            keys = ents[b_idx].astype(np.int64) * ds.dim + f_idx
            vals = orig[b_idx, f_idx]
            vv = None if vorig is None else vorig[b_idx, f_idx]
        nz = vals != 0
        return keys[nz], vals[nz], (None if vv is None else vv[nz])

    def score(self, model: RandomEffectModel) -> torch.Tensor:
        ds = self.dataset
        last = getattr(self, "_last", None)
        if ds.layout == "segmented" and last is not None and last[0] is model:
            # the model just solved: its active-row scores are one forward pass over the block-diagonal data
            # (or, when every entity was solved in its row space, L beta)
            rz = getattr(self, "_rs_scores", None)
            z = rz if rz is not None else ds.seg.glm.matvec(last[1])
            if getattr(ds, "seg_rows_identity", False) and z.numel() == self.data.n_rows:
                out = z.clone()
            else:
                out = torch.zeros(self.data.n_rows, dtype=torch.float64, device=z.device)
                out[ds.seg_rows] = z
            if len(ds.passive_rows):
                pm = np.zeros(self.data.n_rows, dtype=bool)
                pm[ds.passive_rows] = True
                out = out + model.score(self.data, z.device, mask=pm).to(torch.float64)
            return out.to(self.device)
        return model.score(self.data, self.device, mask=ds.score_mask).to(torch.float64)

    def regularization_term_value(self, model: RandomEffectModel) -> float:
        reg, lam = self.opt_config.regularization_context, self.opt_config.regularization_weight
        l1w = reg.l1_weight(lam)
        a, q = model.sum_abs_and_sq(need_abs=l1w != 0)
        return (l1w * a if l1w != 0 else 0.0) + 0.5 * reg.l2_weight(lam) * q


class ShardedRandomEffectCoordinate(Coordinate):
    """Random-effect coordinate under a process group: entities are OWNED by one rank each.

    Construction routes every local sample row of this coordinate's feature shard to the owner of its entity
    (:class:`photon_ml_amd.parallel.sharding.RowRouter`, one all-to-all — SURVEY C8) and builds an ordinary
    :class:`RandomEffectCoordinate` over the received rows. Each update then moves only N-length vectors:
    partial scores forward (C11), new scores backward (C12). The returned :class:`RandomEffectModel` holds the
    owned entities only; save it per rank (``io.model_io.save_game_model`` writes per-rank part files).
    Reference: ``RandomEffectDataSetPartitioner.scala:113-147``, ``RandomEffectCoordinate.scala:103-187``.
    """

    def __init__(self, coordinate_id: str, data: GameData, data_config: RandomEffectDataConfiguration,
                 opt_config: GLMOptimizationConfiguration, task, compute_variance: bool = False, device=None,
                 dtype=torch.float64):
        from ..parallel.sharding import EntityPartitioner, RowRouter, entity_keys
        self.coordinate_id = coordinate_id
        self.data_config = data_config
        self.device = torch.device(device) if device is not None else default_device()
        re_type, shard = data_config.random_effect_type, data_config.feature_shard_id
        ids = np.asarray(data.id_tags[re_type])
        self.route_times = {}
        self.routed_bytes = 0            # bytes of residual / score vectors this rank sent away, last update
        placement = getattr(data, "placement", None)
        if placement is not None and placement.re_type == re_type:
            # rows were placed on their entity owners at ingest (parallel/placement.py): this is the PRIMARY
            # coordinate, every row is already local — no routing at build and none per update
            self.partitioner = placement.partitioner
            self.router = None
            self.recv_data = data
        else:
            t0 = time.perf_counter()
            # entity keys, the partitioner's histograms and the routing permutation all on the device (C8 / C9)
            keys = entity_keys(ids, self.device)
            self.partitioner = EntityPartitioner.build_t(keys)
            self.router = RowRouter(self.partitioner.owner_t(keys))
            del keys
            self._sync()
            self.route_times["partition"] = time.perf_counter() - t0
            self.recv_data = self._route(data, self.router, ids, self.route_times)
        self.inner = RandomEffectCoordinate(coordinate_id, self.recv_data, data_config, opt_config, task,
                                            compute_variance, device, dtype)
        self._val_cache = {}

    def _sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def _route(self, data: GameData, router, ids, times: Optional[dict] = None) -> GameData:
        """Move this coordinate's rows to the owners of their entities (C8): the feature rows stay device tensors
        end to end (device permutation + all-to-all, kept as a :class:`DeviceCSR` for the device dataset build),
        the per-row vectors and integer entity ids as one all-to-all each; string ids as codes plus only the
        distinct names each owner needs (``RowRouter.forward_strings``). ``times``: per-phase seconds."""
        re_type, shard = self.data_config.random_effect_type, self.data_config.feature_shard_id
        dev = self.device
        fwd = lambda a: router.forward(torch.from_numpy(np.ascontiguousarray(a)).to(dev)).cpu().numpy()
        times = {} if times is None else times
        with Timed(f"RE {self.coordinate_id}: route rows to entity owners", log, logging.INFO):
            t0 = time.perf_counter()
            x = router.forward_csr_device(data.shard(shard), dev, times)
            self._sync()
            t1 = time.perf_counter()
            ids = np.asarray(ids)
            recv_ids = fwd(ids.astype(np.int64)) if ids.dtype.kind in "iu" else router.forward_strings(ids)
            tags = {re_type: recv_ids}
            out = GameData(fwd(data.response), {shard: x}, tags, fwd(data.offsets), fwd(data.weights),
                           fwd(data.uids), None)
            t2 = time.perf_counter()
            times.update(rows=t1 - t0, vectors=t2 - t1)
            log.info("RE %s routing: %s", self.coordinate_id, {k: round(v, 3) for k, v in times.items()})
            return out

    @property
    def dataset(self):
        return self.inner.dataset

    @property
    def last_stats(self):
        return self.inner.last_stats

    def solver_routing(self) -> dict:
        return self.inner.solver_routing()

    def set_config(self, opt_config):
        self.inner.set_config(opt_config)

    def initialize_model(self):
        return self.inner.initialize_model()

    @property
    def placed(self) -> bool:
        """True for the primary coordinate of entity-placed data (identity routing)."""
        return self.router is None

    def _off_rank_bytes(self) -> int:
        """Bytes of one fp64 per-row vector this rank sends to other ranks through the router."""
        if self.router is None:
            return 0
        from ..parallel.dist import rank
        return 8 * int(sum(self.router.send_counts) - self.router.send_counts[rank()])

    def update_model(self, model, partial_score: Optional[torch.Tensor] = None):
        # partial scores go to the entity owners on the device (no host staging under RCCL, see RowRouter)
        self.routed_bytes = 0
        if partial_score is None or self.router is None:
            p = None if partial_score is None else partial_score.detach().to(self.device, torch.float64)
        else:
            p = self.router.forward(partial_score.detach().to(self.device, torch.float64))
            self.routed_bytes += self._off_rank_bytes()
        return self.inner.update_model(model, p)

    def score(self, model) -> torch.Tensor:
        s = self.inner.score(model).detach().to(self.device, torch.float64)
        if self.router is None:
            return s
        self.routed_bytes += self._off_rank_bytes()
        return self.router.backward(s)

    def score_validation(self, model, vdata: GameData) -> torch.Tensor:
        """Route validation rows to entity owners once (cached per dataset), score there, route back."""
        from ..parallel.sharding import RowRouter, entity_keys
        key = id(vdata)
        if key not in self._val_cache:
            ids = np.asarray(vdata.id_tags[self.data_config.random_effect_type])
            router = RowRouter(self.partitioner.owner_t(entity_keys(ids, self.device)))
            self._val_cache[key] = (router, self._route(vdata, router, ids))
        router, recv = self._val_cache[key]
        s = model.score(recv, self.device).to(torch.float64)
        return router.backward(s)

    def regularization_term_value(self, model) -> float:
        from ..parallel.dist import all_reduce_scalar
        return all_reduce_scalar(self.inner.regularization_term_value(model))
