"""Generalized linear model classes and coefficients.

Reference: ``photon-lib/.../model/Coefficients.scala:31-168`` (means + optional variances, ``computeScore``),
``photon-api/.../supervised/model/GeneralizedLinearModel.scala:33-178`` and the concrete models
(``classification/LogisticRegressionModel.scala``, ``regression/{Linear,Poisson}RegressionModel.scala``,
``classification/SmoothedHingeLossLinearSVMModel.scala``), ``BinaryClassifier.scala`` (threshold 0.5).

Coefficient vectors are fp64 torch tensors (dense) — on device for training, moved to host for IO.
The reference FQCNs are kept as aliases so saved Avro models interoperate (``modelClass`` field).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from ..constants import TaskType

FQCN = {
    TaskType.LOGISTIC_REGRESSION: "com.linkedin.photon.ml.supervised.classification.LogisticRegressionModel",
    TaskType.LINEAR_REGRESSION: "com.linkedin.photon.ml.supervised.regression.LinearRegressionModel",
    TaskType.POISSON_REGRESSION: "com.linkedin.photon.ml.supervised.regression.PoissonRegressionModel",
    TaskType.SMOOTHED_HINGE_LOSS_LINEAR_SVM:
        "com.linkedin.photon.ml.supervised.classification.SmoothedHingeLossLinearSVMModel",
}
LOSS_FQCN = {
    TaskType.LOGISTIC_REGRESSION: "com.linkedin.photon.ml.function.glm.LogisticLossFunction",
    TaskType.LINEAR_REGRESSION: "com.linkedin.photon.ml.function.glm.SquaredLossFunction",
    TaskType.POISSON_REGRESSION: "com.linkedin.photon.ml.function.glm.PoissonLossFunction",
    TaskType.SMOOTHED_HINGE_LOSS_LINEAR_SVM: "com.linkedin.photon.ml.function.svm.SmoothedHingeLossFunction",
}


def task_from_model_class(name: str) -> TaskType:
    short = name.rsplit(".", 1)[-1]
    for t, fq in FQCN.items():
        if fq == name or fq.rsplit(".", 1)[-1] == short:
            return t
    raise ValueError(f"unknown model class {name}")


@dataclass
class Coefficients:
    means: torch.Tensor
    variances: Optional[torch.Tensor] = None

    def __post_init__(self):
        self.means = torch.as_tensor(self.means, dtype=torch.float64)
        if self.variances is not None:
            self.variances = torch.as_tensor(self.variances, dtype=torch.float64)
            if self.variances.shape != self.means.shape:
                raise ValueError("means and variances must have the same shape")

    @property
    def dim(self) -> int:
        return int(self.means.numel())

    def compute_score(self, x) -> torch.Tensor:
        """``x . means`` for a dense vector, dense matrix, scipy CSR or torch tensor."""
        import scipy.sparse as sp
        if sp.issparse(x):
            return torch.from_numpy(np.asarray(x @ self.means.cpu().numpy()).reshape(-1))
        x = torch.as_tensor(x, dtype=torch.float64, device=self.means.device)
        return x @ self.means

    def to(self, device) -> "Coefficients":
        return Coefficients(self.means.to(device), None if self.variances is None else self.variances.to(device))

    def equals(self, other: "Coefficients", tol: float = 1e-12) -> bool:
        if self.dim != other.dim:
            return False
        if not torch.allclose(self.means.cpu(), other.means.cpu(), atol=tol, rtol=0):
            return False
        if (self.variances is None) != (other.variances is None):
            return False
        return self.variances is None or torch.allclose(self.variances.cpu(), other.variances.cpu(), atol=tol,
                                                        rtol=0)

    @staticmethod
    def zeros(dim: int, device="cpu") -> "Coefficients":
        return Coefficients(torch.zeros(dim, dtype=torch.float64, device=device))


class GeneralizedLinearModel:
    task: TaskType = TaskType.NONE

    def __init__(self, coefficients: Coefficients):
        self.coefficients = coefficients

    @property
    def model_class(self) -> str:
        return FQCN[self.task]

    def compute_score(self, x) -> torch.Tensor:
        return self.coefficients.compute_score(x)

    def mean_from_score(self, score: torch.Tensor) -> torch.Tensor:  # link^-1
        raise NotImplementedError

    def compute_mean(self, x, offset=0.0) -> torch.Tensor:
        return self.mean_from_score(self.compute_score(x) + offset)

    def update_coefficients(self, c: Coefficients) -> "GeneralizedLinearModel":
        return type(self)(c)

    def validate_coefficients(self):
        m = self.coefficients.means
        bad = (~torch.isfinite(m)).nonzero().flatten().tolist()
        if bad:
            raise ValueError("Detected invalid coefficients / offset: " +
                             "".join(f"Index [{i}] has value [{float(m[i])}]\n" for i in bad[:20]))

    def __eq__(self, other):
        return type(self) is type(other) and self.coefficients.equals(other.coefficients)

    def __repr__(self):
        return f"{type(self).__name__}(dim={self.coefficients.dim})"


class LogisticRegressionModel(GeneralizedLinearModel):
    task = TaskType.LOGISTIC_REGRESSION
    threshold = 0.5

    def mean_from_score(self, s):
        return torch.sigmoid(torch.as_tensor(s, dtype=torch.float64))

    def predict_class(self, x, offset=0.0, threshold: float = 0.5):
        return (self.compute_mean(x, offset) > threshold).to(torch.float64)


class LinearRegressionModel(GeneralizedLinearModel):
    task = TaskType.LINEAR_REGRESSION

    def mean_from_score(self, s):
        return torch.as_tensor(s, dtype=torch.float64)


class PoissonRegressionModel(GeneralizedLinearModel):
    task = TaskType.POISSON_REGRESSION

    def mean_from_score(self, s):
        return torch.exp(torch.as_tensor(s, dtype=torch.float64))


class SmoothedHingeLossLinearSVMModel(GeneralizedLinearModel):
    task = TaskType.SMOOTHED_HINGE_LOSS_LINEAR_SVM
    threshold = 0.0

    def mean_from_score(self, s):
        return torch.as_tensor(s, dtype=torch.float64)

    def predict_class(self, x, offset=0.0, threshold: float = 0.0):
        return (self.compute_mean(x, offset) > threshold).to(torch.float64)


MODEL_BY_TASK = {
    TaskType.LOGISTIC_REGRESSION: LogisticRegressionModel,
    TaskType.LINEAR_REGRESSION: LinearRegressionModel,
    TaskType.POISSON_REGRESSION: PoissonRegressionModel,
    TaskType.SMOOTHED_HINGE_LOSS_LINEAR_SVM: SmoothedHingeLossLinearSVMModel,
}


def model_for_task(task, coefficients: Coefficients) -> GeneralizedLinearModel:
    return MODEL_BY_TASK[TaskType.parse(task)](coefficients)
