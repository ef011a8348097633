"""Estimator API: GameEstimator (fit), GameTransformer (score), and the legacy GLM lambda-path trainer.

Reference:
  * ``photon-api/.../estimators/GameEstimator.scala:56-753`` — params (training task, input column names,
    coordinate data configurations, update sequence, CD iterations (default 1), normalization contexts,
    compute variance (false), tree aggregate depth (1), validation evaluators, warm start (true)); ``fit`` trains
    one GAME model per optimisation configuration in sequence, warm-starting from the previous one.
  * ``photon-api/.../transformers/GameTransformer.scala:38-308`` — score a dataset with a GameModel, optionally
    evaluate.
  * ``photon-api/.../ModelTraining.scala:35-234`` — legacy GLM training over a lambda grid sorted DESCENDING,
    each lambda warm-started from the previous model.

Datasets are built ONCE per ``fit`` (device-resident shards / buckets) and reused across configurations; a new
configuration only swaps the optimisation problem of each coordinate.
"""
from __future__ import annotations

import logging
import os
from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..algorithm.coordinate_descent import CoordinateDescent
from ..algorithm.coordinates import FixedEffectCoordinate, RandomEffectCoordinate, ShardedRandomEffectCoordinate
from ..constants import RANDOM_SEED, TaskType
from ..data.game_data import GameData
from ..data.matrix import LabeledData
from ..data.random_effect import FixedEffectDataConfiguration, RandomEffectDataConfiguration
from ..evaluation.evaluators import (build_evaluator, default_validation_evaluator, parse_evaluator_type,
                                     training_loss_evaluator_type)
from ..models.game import GameModel
from ..normalization.context import NormalizationContext, NormalizationType
from ..ops.backend import default_device, make_glm_data
from ..optimization.config import (GLMOptimizationConfiguration, OptimizerConfig, OptimizerType,
                                   RegularizationContext)
from ..optimization.problem import GLMOptimizationProblem
from ..parallel.dist import DistributedGLMData, is_dist
from ..stat.summary import BasicStatisticalSummary

log = logging.getLogger(__name__)

DEFAULT_TREE_AGGREGATE_DEPTH = 1


@dataclass
class GameResult:
    model: GameModel
    evaluations: Optional[list]
    config: Dict[str, GLMOptimizationConfiguration]


class GameEstimator:
    def __init__(self, device=None, precision: str = "f64"):
        self.training_task: Optional[TaskType] = None
        self.coordinate_data_configurations: "OrderedDict[str, object]" = OrderedDict()
        self.coordinate_update_sequence: Optional[List[str]] = None
        self.coordinate_descent_iterations = 1
        self.coordinate_normalization_contexts: Dict[str, NormalizationContext] = {}
        self.compute_variance = False
        self.tree_aggregate_depth = DEFAULT_TREE_AGGREGATE_DEPTH
        self.validation_evaluators: Optional[List[str]] = None
        self.use_warm_start = True
        self.device = torch.device(device) if device is not None else default_device()
        self.precision = precision
        self.event_callback = None
        self.coordinates = None
        self.history: List[list] = []
        self.checkpoint_directory: Optional[str] = None
        self.resume = False

    # fluent setters mirroring Spark ML Params ------------------------------------------------------------
    def set_training_task(self, t):
        self.training_task = TaskType.parse(t)
        return self

    def set_coordinate_data_configurations(self, cfgs):
        self.coordinate_data_configurations = OrderedDict(cfgs)
        return self

    def set_coordinate_update_sequence(self, seq):
        self.coordinate_update_sequence = list(seq)
        return self

    def set_coordinate_descent_iterations(self, n: int):
        if n <= 0:
            raise ValueError("coordinate descent iterations must be > 0")
        self.coordinate_descent_iterations = n
        return self

    def set_coordinate_normalization_contexts(self, ctxs):
        self.coordinate_normalization_contexts = dict(ctxs)
        return self

    def set_compute_variance(self, b: bool):
        self.compute_variance = bool(b)
        return self

    def set_tree_aggregate_depth(self, d: int):
        if d <= 0:
            raise ValueError("tree aggregate depth must be > 0")
        self.tree_aggregate_depth = d
        # the reduction-shape knob maps to the RCCL all-reduce algorithm (depth >= 2 -> tree, else RCCL's choice)
        from ..parallel.dist import set_allreduce_algo
        set_allreduce_algo(tree_depth=d)
        return self

    def set_validation_evaluators(self, evs):
        self.validation_evaluators = [e if isinstance(e, str) else e.name for e in evs]
        return self

    def set_entity_placement(self, coordinate: Optional[str] = "auto"):
        """Multi-GPU only: place every training row on the owner of its entity in one random-effect coordinate at
        the start of ``fit`` (parallel/placement.py), so that coordinate needs no per-update routing and the fixed
        effects train on the placed rows. ``"auto"``: the first random-effect coordinate of the update sequence;
        None: no placement (every random-effect coordinate routes its rows)."""
        self.entity_placement = coordinate
        return self

    def set_warm_start(self, b: bool):
        self.use_warm_start = bool(b)
        return self

    def set_initial_model(self, model: Optional[GameModel]):
        """Start the first configuration from a saved model (e.g. ``load_game_model``) instead of zeros; the
        reference has no such option (warm start only in-process)."""
        self.initial_model = model
        return self

    def set_checkpoint_directory(self, directory: Optional[str], resume: bool = False):
        """Checkpoint coordinate descent after every coordinate update (one state file per configuration and
        rank); with ``resume`` an interrupted fit continues where it stopped (see utils/checkpoint.py)."""
        self.checkpoint_directory = directory
        self.resume = bool(resume)
        return self

    # ----------------------------------------------------------------------------------------------------
    def validate_params(self):
        if self.training_task is None:
            raise ValueError("training task is required")
        if not self.coordinate_data_configurations:
            raise ValueError("coordinate data configurations are required")
        seq = self.coordinate_update_sequence or list(self.coordinate_data_configurations)
        missing = [c for c in seq if c not in self.coordinate_data_configurations]
        if missing:
            raise ValueError(f"coordinates {missing} in the update sequence have no data configuration")
        return seq

    def _build_coordinates(self, data: GameData, first_cfg: Dict[str, GLMOptimizationConfiguration], seq):
        from ..ops.warmup import runtime_warmup
        from ..utils.timing import Timed
        dev = self.device if self.device is not None else default_device()
        with Timed("Device runtime warm-up (first kernel launches of the process)"):
            self.runtime_warmup_s = runtime_warmup(dev)
        coords = OrderedDict()
        # the first random-effect shard built after a fixed-effect coordinate is copied to the device while the GPU
        # builds the fixed-effect layout (a host CSR shard no fixed effect reads; GPU only)
        fe_shards = {dc.feature_shard_id for dc in self.coordinate_data_configurations.values()
                     if not isinstance(dc, RandomEffectDataConfiguration)}
        seen_fe = False
        for cid in seq:
            dc = self.coordinate_data_configurations[cid]
            if not isinstance(dc, RandomEffectDataConfiguration):
                seen_fe = True
            elif seen_fe and dc.feature_shard_id not in fe_shards:
                data.prefetch_shard(dc.feature_shard_id, dev)
                break
        for cid in seq:
            dc = self.coordinate_data_configurations[cid]
            oc = first_cfg[cid]
            if isinstance(dc, RandomEffectDataConfiguration):
                cls = ShardedRandomEffectCoordinate if is_dist() else RandomEffectCoordinate
                coords[cid] = cls(cid, data, dc, oc, self.training_task, self.compute_variance, self.device)
            else:
                coords[cid] = FixedEffectCoordinate(cid, data, dc, oc, self.training_task,
                                                    self.coordinate_normalization_contexts.get(cid),
                                                    self.compute_variance, self.device, self.precision)
        return coords

    def _place(self, data: GameData, seq) -> GameData:
        """Entity-aligned placement of the training rows (see :meth:`set_entity_placement`)."""
        want = getattr(self, "entity_placement", "auto")
        if not is_dist() or want is None:
            return data
        re_cids = [c for c in seq if isinstance(self.coordinate_data_configurations[c], RandomEffectDataConfiguration)]
        cid = re_cids[0] if want == "auto" and re_cids else want
        if cid not in re_cids:
            return data
        from ..parallel.placement import place_rows_by_entity
        re_type = self.coordinate_data_configurations[cid].random_effect_type
        if getattr(getattr(data, "placement", None), "re_type", None) == re_type:
            return data
        dev = self.device if self.device is not None else default_device()
        return place_rows_by_entity(data, re_type, dev)

    def _validation_evaluators(self, validation: GameData):
        names = self.validation_evaluators or [default_validation_evaluator(self.training_task)]
        return [build_evaluator(parse_evaluator_type(n), validation.response, validation.offsets, validation.weights,
                                validation.id_tags) for n in names]

    def fit(self, data: GameData, validation: Optional[GameData],
            configurations: Sequence[Dict[str, GLMOptimizationConfiguration]]) -> List[GameResult]:
        seq = self.validate_params()
        if not configurations:
            raise ValueError("at least one optimization configuration is required")
        for cfg in configurations:
            missing = [c for c in seq if c not in cfg]
            if missing:
                raise ValueError(f"optimization configuration missing coordinates {missing}")
        data = self._place(data, seq)
        self.coordinates = self._build_coordinates(data, configurations[0], seq)
        train_eval = build_evaluator(training_loss_evaluator_type(self.training_task), data.response, data.offsets,
                                     data.weights)
        val_evals = self._validation_evaluators(validation) if validation is not None else []
        if val_evals:
            # random-guess baseline of every validation metric (GameEstimator.scala:496-500)
            gen = torch.Generator().manual_seed(RANDOM_SEED)
            rnd = torch.rand(validation.n_rows, generator=gen, dtype=torch.float64)
            for e in val_evals:
                log.info("Random guessing based baseline evaluation metric for %s: %s", e.name,
                         e.evaluate(rnd))
        results, prev = [], getattr(self, "initial_model", None)
        for i, cfg in enumerate(configurations):
            for cid, c in self.coordinates.items():
                c.set_config(cfg[cid])
            cd = CoordinateDescent(self.coordinates, train_eval, validation, val_evals,
                                   event_callback=self.event_callback)
            ck, tag = None, ""
            if self.checkpoint_directory:
                from ..utils.checkpoint import Checkpointer
                import json as _json
                ck = Checkpointer(self.checkpoint_directory, f"cd-state-{i}")
                tag = _json.dumps({c: cfg[c].to_json() for c in sorted(cfg)}, sort_keys=True)
                if not self.resume and ck.exists():
                    os.remove(ck.path)
            model, evals = cd.run(self.coordinate_descent_iterations, prev if (self.use_warm_start or i == 0) else None, ck,
                                  tag)
            self.history.append(cd.history)
            results.append(GameResult(model, evals, cfg))
            if self.use_warm_start:
                prev = model
        return results


class GameTransformer:
    def __init__(self, model: GameModel, validation_evaluators: Optional[Sequence[str]] = None, device=None):
        """``device`` defaults to the current GPU (the HIP scoring kernels, K5/K6) and to the CPU without one."""
        self.model = model
        self.validation_evaluators = list(validation_evaluators or [])
        self.device = torch.device(device) if device is not None else default_device()

    def transform(self, data: GameData):
        """Return (scores WITHOUT offsets, evaluations or None)."""
        return self._evaluate(data, self.model.score(data, self.device))

    def _evaluate(self, data: GameData, scores):
        evals = None
        if self.validation_evaluators:
            evals = []
            for n in self.validation_evaluators:
                e = build_evaluator(parse_evaluator_type(n), data.response, data.offsets, data.weights, data.id_tags)
                evals.append((e, e.evaluate(scores)))
        return scores, evals

    def transform_spilled(self, data: GameData, path: str, chunk_rows: int = 1 << 24):
        """:meth:`transform` for score sets that should not stay resident (``--spill-scores-to-disk``; the
        reference persists the scores RDD with MEMORY_AND_DISK, ``GameScoringDriver.scala:55-70``): rows are
        scored ``chunk_rows`` at a time on the device and each chunk goes straight into a memory-mapped fp64 file
        at ``path`` (``.npy``), so device memory holds one chunk of scores and the host keeps only pages the OS
        chooses to. Returns (CPU tensor over the mapped file, evaluations)."""
        n = data.n_rows
        mm = np.lib.format.open_memmap(path, mode="w+", dtype=np.float64, shape=(n,))
        for lo in range(0, n, chunk_rows):
            hi = min(n, lo + chunk_rows)
            sub = data if (lo == 0 and hi == n) else data.subset(np.arange(lo, hi))
            mm[lo:hi] = self.model.score(sub, self.device).detach().to("cpu", torch.float64).numpy()
            del sub
        mm.flush()
        return self._evaluate(data, torch.from_numpy(mm))


# --------------------------------------------------------------------------------------------------------------
def train_generalized_linear_model(data: LabeledData, task, optimizer_type="LBFGS",
                                   regularization: RegularizationContext = RegularizationContext("L2"),
                                   regularization_weights: Sequence[float] = (10.0,),
                                   normalization: Optional[NormalizationContext] = None, max_iterations: int = 80,
                                   tolerance: float = 1e-6, constraint_map=None, warm_start_models=None,
                                   use_warm_start: bool = True, compute_variance: bool = False, device=None,
                                   precision: str = "f64", glm_data=None, feature_sharded: bool = False):
    """ModelTraining.trainGeneralizedLinearModel -> list of (lambda, model, tracker), lambdas DESCENDING.

    ``feature_sharded``: under a process group, shard the optimizer state over features instead of replicating
    it (``parallel/feature_sharding.py``; for models too large to replicate)."""
    device = torch.device(device) if device is not None else default_device()
    gdata = glm_data if glm_data is not None else make_glm_data(data, device, precision)
    view = DistributedGLMData(gdata) if is_dist() and not feature_sharded else gdata
    lams = sorted(regularization_weights, reverse=True)
    out = []
    prev = None
    for lam in lams:
        cfg = GLMOptimizationConfiguration(OptimizerConfig(optimizer_type, max_iterations, tolerance, constraint_map),
                                           regularization, lam)
        prob = GLMOptimizationProblem(cfg, task, normalization, compute_variance, feature_sharded=feature_sharded)
        init = None
        if warm_start_models and lam in warm_start_models:
            init = warm_start_models[lam]
        elif use_warm_start and prev is not None:
            init = prev
        model = prob.run(view, init, dim=gdata.dim)
        out.append((lam, model, prob.tracker))
        prev = model
    return out
