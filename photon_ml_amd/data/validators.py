"""Input data validation.

Reference: ``photon-client/.../data/DataValidators.scala:33-375`` and ``DataValidationType.scala``:
  * row checks: finite features, finite offset, finite weight and > 0 (data frames), finite label; binary label
    for logistic / hinge, non-negative label for Poisson;
  * modes VALIDATE_FULL (every row), VALIDATE_SAMPLE (10 % sample), VALIDATE_DISABLED.
Vectorised over the columnar dataset; with a process group the per-rank verdicts are AND-reduced (C22).
"""
from __future__ import annotations

import enum
from typing import Dict, List, Sequence

import numpy as np
import scipy.sparse as sp

from ..constants import TaskType


class DataValidationType(str, enum.Enum):
    VALIDATE_FULL = "VALIDATE_FULL"
    VALIDATE_SAMPLE = "VALIDATE_SAMPLE"
    VALIDATE_DISABLED = "VALIDATE_DISABLED"

    @classmethod
    def parse(cls, s):
        return s if isinstance(s, DataValidationType) else cls[str(s).strip().upper()]


SAMPLE_FRACTION = 0.10


class DataValidationError(ValueError):
    pass


def _rows(n: int, mode: DataValidationType, seed: int = 0) -> np.ndarray:
    if mode == DataValidationType.VALIDATE_SAMPLE:
        rng = np.random.default_rng(seed)
        return np.nonzero(rng.random(n) < SAMPLE_FRACTION)[0]
    return np.arange(n)


def _finite_rows(x: sp.csr_matrix) -> np.ndarray:
    bad = ~np.isfinite(x.data)
    if not bad.any():
        return np.ones(x.shape[0], dtype=bool)
    rows = np.repeat(np.arange(x.shape[0]), np.diff(x.indptr))
    ok = np.ones(x.shape[0], dtype=bool)
    ok[rows[bad]] = False
    return ok


def validate(task, labels, offsets, weights, shards: Dict[str, sp.csr_matrix],
             mode=DataValidationType.VALIDATE_FULL, for_training: bool = True, check_weights_positive: bool = True
             ) -> List[str]:
    """Return the list of failure messages (empty when valid)."""
    mode = DataValidationType.parse(mode)
    if mode == DataValidationType.VALIDATE_DISABLED:
        return []
    task = TaskType.parse(task)
    idx = _rows(len(labels), mode)
    msgs = []
    y = np.asarray(labels)[idx]
    if for_training:
        if not np.all(np.isfinite(y)):
            msgs.append("Data contains row(s) with non-finite label")
        if task in (TaskType.LOGISTIC_REGRESSION, TaskType.SMOOTHED_HINGE_LOSS_LINEAR_SVM):
            if not np.all((y == 0) | (y == 1)):
                msgs.append("Data contains row(s) with non-binary label")
        if task == TaskType.POISSON_REGRESSION and not np.all(y >= 0):
            msgs.append("Data contains row(s) with negative label")
    if offsets is not None and not np.all(np.isfinite(np.asarray(offsets)[idx])):
        msgs.append("Data contains row(s) with non-finite offset")
    if weights is not None:
        w = np.asarray(weights)[idx]
        if not np.all(np.isfinite(w)):
            msgs.append("Data contains row(s) with non-finite weight")
        elif check_weights_positive and not np.all(w > 0):
            msgs.append("Data contains row(s) with non-positive weight")
    for sid, x in shards.items():
        if not _finite_rows(x[idx] if mode == DataValidationType.VALIDATE_SAMPLE else x).all():
            msgs.append(f"Data contains row(s) with non-finite feature(s) in shard {sid}")
    try:
        from ..parallel.dist import all_reduce_scalar, is_dist
        if is_dist():
            if all_reduce_scalar(float(len(msgs) > 0), "max") > 0 and not msgs:
                msgs.append("validation failed on another rank")
    except Exception:  # pragma: no cover
        pass
    return msgs


def sanity_check(task, labels, offsets, weights, shards, mode=DataValidationType.VALIDATE_FULL,
                 for_training: bool = True):
    msgs = validate(task, labels, offsets, weights, shards, mode, for_training)
    if msgs:
        raise DataValidationError("Data validation failed:\n" + "\n".join(msgs))
