"""GAME hyper-parameter evaluation function: regularisation weights <-> search vector.

Reference: ``photon-client/.../hyperparameter/GameEstimatorEvaluationFunction.scala:30-140`` — the vector holds one
regularisation weight per coordinate, coordinates sorted by id; evaluating a vector re-fits the estimator with that
configuration and returns the first validation evaluator's value.

Deliberate difference: the search runs in ``log10(λ)`` space by default (``scale="LOG"``) — the reference searches
λ linearly over ``[1e-4, 1e4]`` which puts almost every candidate above 1; ``scale="LINEAR"`` restores it.
"""
from __future__ import annotations

import math
from typing import Dict, List

import numpy as np

from ..optimization.config import GLMOptimizationConfiguration
from .search import DoubleRange, EvaluationFunction


class GameEstimatorEvaluationFunction(EvaluationFunction):
    def __init__(self, estimator, base_config: Dict[str, GLMOptimizationConfiguration], data, validation_data,
                 scale: str = "LOG"):
        self.estimator = estimator
        self.base = sorted(base_config.items())
        self.data = data
        self.validation = validation_data
        self.scale = scale.upper()
        if self.scale not in ("LOG", "LINEAR"):
            raise ValueError(f"unknown tuning scale {scale}")
        self.higher_is_better = True
        self.evaluator = None

    @property
    def num_params(self) -> int:
        return len(self.base)

    def search_ranges(self, lam_range: DoubleRange) -> List[DoubleRange]:
        if self.scale == "LOG":
            if lam_range.start <= 0:
                raise ValueError("log-scale tuning needs a positive λ range")
            r = DoubleRange(math.log10(lam_range.start), math.log10(lam_range.end))
        else:
            r = lam_range
        return [r] * self.num_params

    def _to_lam(self, v):
        return 10.0 ** v if self.scale == "LOG" else v

    def _from_lam(self, lam):
        return math.log10(max(lam, 1e-300)) if self.scale == "LOG" else lam

    def vector_to_configuration(self, v) -> Dict[str, GLMOptimizationConfiguration]:
        v = np.asarray(v, dtype=np.float64)
        if v.size != self.num_params:
            raise ValueError(f"Configuration dimension mismatch; {self.num_params} != {v.size}")
        return {cid: cfg.with_reg_weight(float(self._to_lam(x))) for (cid, cfg), x in zip(self.base, v)}

    def configuration_to_vector(self, config: Dict[str, GLMOptimizationConfiguration]) -> np.ndarray:
        if set(config) != {c for c, _ in self.base}:
            raise ValueError("Configuration coordinates do not match the base configuration")
        return np.array([self._from_lam(config[cid].regularization_weight) for cid, _ in self.base])

    def __call__(self, candidate):
        cfg = self.vector_to_configuration(candidate)
        result = self.estimator.fit(self.data, self.validation, [cfg])[0]
        return self.get_evaluation_value(result), result

    def vectorize_params(self, observation) -> np.ndarray:
        return self.configuration_to_vector(observation.config)

    def get_evaluation_value(self, observation) -> float:
        if not observation.evaluations:
            raise ValueError("Can't extract evaluation value from a GAME result with no evaluations")
        ev, value = observation.evaluations[0]
        self.evaluator = ev
        self.higher_is_better = ev.higher_is_better
        return float(value)
