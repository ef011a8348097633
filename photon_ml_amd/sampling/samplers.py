"""Down-samplers for fixed-effect training (K20).

Reference: ``photon-lib/.../sampler/BinaryClassificationDownSampler.scala:32-69`` (keep every positive, keep each
negative with probability ``rate`` and divide its weight by ``rate``), ``DefaultDownSampler.scala:27-41`` (uniform
sampling without replacement, weights unchanged) and the per-task choice in
``photon-api/.../estimators/GameEstimator.scala:644-656``.

The samplers return a new WEIGHT vector (0 = dropped). On the device path the data never moves: a dropped row
simply carries zero weight for this coordinate update, so no compaction/re-layout of the HBM streams is needed;
the weights are rewritten in place by ``downsample_kernel`` (``ops/csrc/game_kernels.hip``, K20). The uniform of a
row is a counter-based hash of (seed, global row id) — splitmix64, top 53 bits — computed identically here on the
host, so the CPU path, the GPU path and every rank of a data-parallel job draw the same sample. Seeds are
deterministic (``MathConst.RANDOM_SEED`` by default) as in the reference.
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from ..constants import POSITIVE_RESPONSE_THRESHOLD, RANDOM_SEED, TaskType

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = (x + np.uint64(0x9E3779B97F4A7C15)) & _M64
        x = ((x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
        x = ((x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
        return x ^ (x >> np.uint64(31))


def row_uniforms(seed: int, row_ids: np.ndarray) -> np.ndarray:
    """U[0, 1) of each row: (splitmix64(seed ^ splitmix64(row id)) >> 11) * 2^-53 (bitwise = the HIP kernel)."""
    ids = np.asarray(row_ids, dtype=np.int64).astype(np.uint64)
    h = _splitmix64(np.uint64(seed & 0xFFFFFFFFFFFFFFFF) ^ _splitmix64(ids))
    return (h >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


class DownSampler:
    def __init__(self, rate: float, seed: int = RANDOM_SEED):
        if not (0.0 < rate < 1.0):
            raise ValueError(f"Invalid down-sampling rate {rate}; must be in (0, 1)")
        self.rate = float(rate)
        self.seed = int(seed)

    binary = False

    def sample_weights(self, labels, weights, row_ids: Optional[np.ndarray] = None) -> np.ndarray:
        """Host weights; ``row_ids`` = global row ids (default 0..n-1)."""
        n = len(labels)
        u = row_uniforms(self.seed, np.arange(n) if row_ids is None else row_ids)
        w = np.asarray(weights, dtype=np.float64)
        if self.binary:
            pos = np.asarray(labels, dtype=np.float64) >= POSITIVE_RESPONSE_THRESHOLD
            return np.where(pos, w, np.where(u < self.rate, w / self.rate, 0.0))
        return np.where(u < self.rate, w, 0.0)

    def sample_weights_device(self, labels, weights, row_ids=None, out=None):
        """The same weights computed on the device (``downsample_kernel``), written into ``out`` if given."""
        from ..ops.native import downsample_weights
        return downsample_weights(labels, weights, self.rate, self.binary, self.seed, row_ids, out)


class BinaryClassificationDownSampler(DownSampler):
    """Keep every positive; keep a negative with probability ``rate`` and divide its weight by ``rate``."""
    binary = True


class DefaultDownSampler(DownSampler):
    """Keep each row with probability ``rate``, weights unchanged."""
    binary = False


def down_sampler_for_task(task, rate: float, seed: int = RANDOM_SEED) -> DownSampler:
    task = TaskType.parse(task)
    if task in (TaskType.LOGISTIC_REGRESSION, TaskType.SMOOTHED_HINGE_LOSS_LINEAR_SVM):
        return BinaryClassificationDownSampler(rate, seed)
    return DefaultDownSampler(rate, seed)
