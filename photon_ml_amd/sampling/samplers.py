"""Down-samplers for fixed-effect training (K20).

Reference: ``photon-lib/.../sampler/BinaryClassificationDownSampler.scala:32-69`` (keep every positive, keep each
negative with probability ``rate`` and divide its weight by ``rate``), ``DefaultDownSampler.scala:27-41`` (uniform
sampling without replacement, weights unchanged) and the per-task choice in
``photon-api/.../estimators/GameEstimator.scala:644-656``.

The samplers return a new WEIGHT vector (0 = dropped). On the device path the data never moves: a dropped row
simply carries zero weight for this coordinate update, so no compaction/re-layout of the HBM streams is needed.
Seeds are deterministic (``MathConst.RANDOM_SEED`` by default) as in the reference.
"""
from __future__ import annotations

import numpy as np

from ..constants import POSITIVE_RESPONSE_THRESHOLD, RANDOM_SEED, TaskType


class DownSampler:
    def __init__(self, rate: float, seed: int = RANDOM_SEED):
        if not (0.0 < rate < 1.0):
            raise ValueError(f"Invalid down-sampling rate {rate}; must be in (0, 1)")
        self.rate = float(rate)
        self.seed = int(seed)

    def sample_weights(self, labels: np.ndarray, weights: np.ndarray) -> np.ndarray:  # pragma: no cover
        raise NotImplementedError


class BinaryClassificationDownSampler(DownSampler):
    def sample_weights(self, labels, weights):
        rng = np.random.default_rng(self.seed)
        u = rng.random(len(labels))
        pos = np.asarray(labels) >= POSITIVE_RESPONSE_THRESHOLD
        keep_neg = u < self.rate
        w = np.asarray(weights, dtype=np.float64)
        return np.where(pos, w, np.where(keep_neg, w / self.rate, 0.0))


class DefaultDownSampler(DownSampler):
    def sample_weights(self, labels, weights):
        rng = np.random.default_rng(self.seed)
        keep = rng.random(len(labels)) < self.rate
        return np.where(keep, np.asarray(weights, dtype=np.float64), 0.0)


def down_sampler_for_task(task, rate: float, seed: int = RANDOM_SEED) -> DownSampler:
    task = TaskType.parse(task)
    if task in (TaskType.LOGISTIC_REGRESSION, TaskType.SMOOTHED_HINGE_LOSS_LINEAR_SVM):
        return BinaryClassificationDownSampler(rate, seed)
    return DefaultDownSampler(rate, seed)
