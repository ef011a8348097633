"""Down-samplers for fixed-effect training (K20).

Reference: ``photon-lib/.../sampler/BinaryClassificationDownSampler.scala:32-69`` (keep every positive, keep each
negative with probability ``rate`` and divide its weight by ``rate``), ``DefaultDownSampler.scala:27-41`` (uniform
sampling without replacement, weights unchanged) and the per-task choice in
``photon-api/.../estimators/GameEstimator.scala:644-656``.

The samplers return a new WEIGHT vector (0 = dropped). On the device path the data never moves: a dropped row
simply carries zero weight for this coordinate update, so no compaction/re-layout of the HBM streams is needed;
the weights are rewritten in place by ``downsample_kernel`` (``ops/csrc/game_kernels.hip``, K20). The uniform of a
row is a counter-based hash of (seed, global row id) — splitmix64, top 53 bits — computed identically here on the
host, so the CPU path, the GPU path and every rank of a data-parallel job draw the same sample.

Seeds follow the reference: every down-sampling call draws a FRESH seed from one process-wide
``java.util.Random(MathConst.RANDOM_SEED)`` sequence (``DownSampler.scala:38-46``: ``random.nextLong()``), so every
fixed-effect update trains on a different sample, and the sequence of seeds is the reference's bit for bit
(:class:`JavaRandom`; the per-row draws themselves are this framework's counter-based hash, not Java's LCG per
Spark partition). Every rank runs the same updates in the same order, so the ranks of a data-parallel job draw
the same seeds.
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


class JavaRandom:
    """``java.util.Random``'s 48-bit LCG (``nextLong`` only): the seed source of the reference's samplers."""
    _MULT, _ADD, _MASK = 0x5DEECE66D, 0xB, (1 << 48) - 1

    def __init__(self, seed: int):
        self._s = (int(seed) ^ self._MULT) & self._MASK

    def _next(self, bits: int) -> int:
        self._s = (self._s * self._MULT + self._ADD) & self._MASK
        v = self._s >> (48 - bits)
        return v - (1 << bits) if v >= 1 << (bits - 1) else v     # Java int (signed 32-bit)

    def next_long(self) -> int:
        v = ((self._next(32) << 32) + self._next(32)) & 0xFFFFFFFFFFFFFFFF
        return v - (1 << 64) if v >= 1 << 63 else v


_SEEDS = JavaRandom(RANDOM_SEED)


def next_seed() -> int:
    """The next down-sampling seed of the process-wide sequence (``DownSampler.getSeed``)."""
    return _SEEDS.next_long()


def reset_seed_sequence(seed: int = RANDOM_SEED):
    """Restart the seed sequence (a fresh process in the reference; tests)."""
    global _SEEDS
    _SEEDS = JavaRandom(seed)


def seed_state() -> int:
    """Position of the process-wide seed sequence (the LCG's 48-bit word): stored in GAME checkpoints so a resumed
    run draws the same down-sampling seeds as an uninterrupted one."""
    return int(_SEEDS._s)


def set_seed_state(state: int):
    """Restore a position saved by :func:`seed_state` (checkpoint resume)."""
    _SEEDS._s = int(state) & JavaRandom._MASK


class DownSampler:
    def __init__(self, rate: float, seed: Optional[int] = None):
        """``seed``: a fixed seed for every call (tests); None = a fresh seed per call from the process-wide
        reference sequence (:func:`next_seed`)."""
        if not (0.0 < rate < 1.0):
            raise ValueError(f"Invalid down-sampling rate {rate}; must be in (0, 1)")
        self.rate = float(rate)
        self.fixed_seed = None if seed is None else int(seed)
        self.seed = self.fixed_seed if seed is not None else None   # seed of the last draw

    binary = False

    def draw_seed(self) -> int:
        """Seed of one down-sampling call (a new draw per call unless the sampler has a fixed seed)."""
        self.seed = self.fixed_seed if self.fixed_seed is not None else next_seed()
        return self.seed

    def sample_weights(self, labels, weights, row_ids: Optional[np.ndarray] = None,
                       seed: Optional[int] = None) -> np.ndarray:
        """Host weights; ``row_ids`` = global row ids (default 0..n-1); ``seed`` default: a new draw."""
        n = len(labels)
        seed = self.draw_seed() if seed is None else seed
        u = row_uniforms(seed, np.arange(n) if row_ids is None else row_ids)
        w = np.asarray(weights, dtype=np.float64)
        if self.binary:
            pos = np.asarray(labels, dtype=np.float64) >= POSITIVE_RESPONSE_THRESHOLD
            return np.where(pos, w, np.where(u < self.rate, w / self.rate, 0.0))
        return np.where(u < self.rate, w, 0.0)

    def sample_weights_device(self, labels, weights, row_ids=None, out=None, seed: Optional[int] = None):
        """The same weights computed on the device (``downsample_kernel``), written into ``out`` if given."""
        from ..ops.native import downsample_weights
        seed = self.draw_seed() if seed is None else seed
        return downsample_weights(labels, weights, self.rate, self.binary, seed, row_ids, out)


class BinaryClassificationDownSampler(DownSampler):
    """Keep every positive; keep a negative with probability ``rate`` and divide its weight by ``rate``."""
    binary = True


class DefaultDownSampler(DownSampler):
    """Keep each row with probability ``rate``, weights unchanged."""
    binary = False


def down_sampler_for_task(task, rate: float, seed: Optional[int] = None) -> DownSampler:
    task = TaskType.parse(task)
    if task in (TaskType.LOGISTIC_REGRESSION, TaskType.SMOOTHED_HINGE_LOSS_LINEAR_SVM):
        return BinaryClassificationDownSampler(rate, seed)
    return DefaultDownSampler(rate, seed)
