"""GLM optimisation problems: objective + optimizer + model construction (+ variances).

Reference: ``photon-api/.../optimization/GeneralizedLinearOptimizationProblem.scala:39-174`` (create the model in
the ORIGINAL space from transformed-space coefficients; regularisation term value = L1 part (OWL-QN weight) +
L2 part), ``DistributedOptimizationProblem.scala:43-203`` (variances = 1/(Hdiag + EPSILON), λ updates,
``runWithSampling``) and ``SingleNodeOptimizationProblem.scala``. One class serves the distributed and the
single-node case: the data backend decides where the aggregation runs.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from ..constants import EPSILON, TaskType
from ..function.losses import loss_for_task
from ..function.objective import GLMObjective
from ..models.glm import Coefficients, GeneralizedLinearModel, model_for_task
from ..normalization.context import NormalizationContext, no_normalization
from .config import GLMOptimizationConfiguration, build_optimizer
from .lbfgs import OWLQN


class GLMOptimizationProblem:
    def __init__(self, config: GLMOptimizationConfiguration, task, normalization: Optional[NormalizationContext] = None,
                 compute_variance: bool = False, track_state: bool = True, feature_sharded: bool = False):
        self.config = config
        # optimizer state sharded over features across the process group (parallel/feature_sharding.py); the
        # data passed to run() is then this rank's row shard, not a DistributedGLMData wrapper
        self.feature_sharded = feature_sharded
        self.checkpointer, self.checkpoint_every = None, 1
        self.task = TaskType.parse(task)
        self.loss = loss_for_task(self.task)
        self.normalization = normalization or no_normalization()
        self.compute_variance = compute_variance
        self.track_state = track_state
        reg = config.regularization_context
        lam = config.regularization_weight
        self.objective = GLMObjective(self.loss, reg.l2_weight(lam), self.normalization)
        self.optimizer = build_optimizer(config.optimizer_config, self.normalization, reg, lam, track_state)

    def update_regularization_weight(self, lam: float):
        reg = self.config.regularization_context
        self.config = self.config.with_reg_weight(lam)
        self.objective.l2_weight = reg.l2_weight(lam)
        if isinstance(self.optimizer, OWLQN):
            self.optimizer.l1_weight = reg.l1_weight(lam)

    @property
    def tracker(self):
        return self.optimizer.tracker

    def _device_of(self, data):
        return getattr(data, "device", torch.device("cpu"))

    def run(self, data, initial: Optional[GeneralizedLinearModel] = None, dim: Optional[int] = None
            ) -> GeneralizedLinearModel:
        dev = self._device_of(data)
        d = dim if dim is not None else data.dim
        w0 = (initial.coefficients.means.to(dev, torch.float64) if initial is not None
              else torch.zeros(d, dtype=torch.float64, device=dev))
        if self.feature_sharded:
            return self._run_feature_sharded(data, w0)
        if self.optimizer.needs_hessian and hasattr(data, "track_hessian"):
            data.track_hessian = True
        if self.checkpointer is not None:
            w_t = self._optimize_checkpointed(data, w0)
        else:
            w_t, _ = self.optimizer.optimize(self.objective, data, w0)
        variances = None
        if self.compute_variance and self.loss.twice_differentiable:
            hd = self.objective.hessian_diagonal(data, w_t)
            variances = self.normalization.model_to_original_space(1.0 / (hd + EPSILON))
        means = self.normalization.model_to_original_space(w_t)
        model = model_for_task(self.task, Coefficients(means.detach(), None if variances is None else variances))
        model.validate_coefficients()
        return model

    def enable_checkpointing(self, checkpointer, every: int = 1):
        """Save the optimizer state every ``every`` iterations (and resume from an existing checkpoint)."""
        self.checkpointer, self.checkpoint_every = checkpointer, max(1, int(every))
        return self

    def _optimize_checkpointed(self, data, w0):
        opt = self.optimizer
        if not self.checkpointer.load_optimizer(opt, device=w0.device):
            opt.start(self.objective, data, w0)
        while not opt.is_done():
            opt.step(self.objective, data)
            if opt.current.iter % self.checkpoint_every == 0:
                self.checkpointer.save_optimizer(opt)
        if opt.tracker is not None:
            opt.tracker.convergence_reason = opt.convergence_reason()
        return opt.current.coefficients

    def _run_feature_sharded(self, data, w0: torch.Tensor) -> GeneralizedLinearModel:
        from ..parallel.feature_sharding import optimize_feature_sharded
        local = getattr(data, "local", data)
        reg = self.config.regularization_context
        opt = build_optimizer(self.config.optimizer_config, None, reg, self.config.regularization_weight,
                              self.track_state)
        self.optimizer = opt
        means, _, sobj = optimize_feature_sharded(opt, self.objective, local, w0, self.normalization)
        variances = None
        if self.compute_variance and self.loss.twice_differentiable:
            from ..parallel.feature_sharding import all_gather_shards
            w_t = self.normalization.model_to_transformed_space(means.clone())
            hd = all_gather_shards(sobj.hessian_diagonal(local, sobj.layout.slice(w_t)), sobj.layout, sobj.group)
            variances = self.normalization.model_to_original_space(1.0 / (hd + EPSILON))
        model = model_for_task(self.task, Coefficients(means.detach(), variances))
        model.validate_coefficients()
        return model

    def regularization_term_value(self, model: GeneralizedLinearModel) -> float:
        w = model.coefficients.means
        reg = self.config.regularization_context
        lam = self.config.regularization_weight
        return reg.l1_weight(lam) * float(w.abs().sum()) + 0.5 * reg.l2_weight(lam) * float(torch.dot(w, w))
