"""Framework-wide constants and enums.

Parity notes (reference = photon-ml):
  * ``EPSILON``, ``RANDOM_SEED``, ``POSITIVE_RESPONSE_THRESHOLD``:
    ``photon-lib/.../constants/MathConst.scala:20-26``.
  * ``TaskType``: ``photon-lib/.../TaskType.scala:20-24``.
  * Feature key delimiter / intercept key: ``photon-client/.../Constants.scala:22-41``.
  * Storage levels do not exist here: data is resident in HBM (or host RAM for the CPU path).
"""
from __future__ import annotations

import enum

EPSILON = 1e-12
RANDOM_SEED = 1234567890
POSITIVE_RESPONSE_THRESHOLD = 0.5

# Feature naming (photon-client Constants.scala)
DELIMITER = "\u0001"
WILDCARD = "*"
INTERCEPT_NAME = "(INTERCEPT)"
INTERCEPT_TERM = ""
INTERCEPT_KEY = INTERCEPT_NAME + DELIMITER + INTERCEPT_TERM

# Minimum |value| written into Avro model files (AvroUtils.scala:192-240)
MODEL_SPARSITY_THRESHOLD = 1e-4


class TaskType(str, enum.Enum):
    LINEAR_REGRESSION = "LINEAR_REGRESSION"
    POISSON_REGRESSION = "POISSON_REGRESSION"
    LOGISTIC_REGRESSION = "LOGISTIC_REGRESSION"
    SMOOTHED_HINGE_LOSS_LINEAR_SVM = "SMOOTHED_HINGE_LOSS_LINEAR_SVM"
    NONE = "NONE"

    @classmethod
    def parse(cls, s: "str | TaskType") -> "TaskType":
        if isinstance(s, TaskType):
            return s
        return cls[str(s).strip().upper()]


def feature_key(name: str, term: str = "") -> str:
    """Build the canonical ``name\\u0001term`` feature key (Utils.getFeatureKey)."""
    return f"{name}{DELIMITER}{term or ''}"


def split_feature_key(key: str) -> tuple[str, str]:
    if DELIMITER in key:
        n, t = key.split(DELIMITER, 1)
        return n, t
    return key, ""
