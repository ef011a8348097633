"""Optimisation configuration: regularisation context, optimizer config, factory, coordinate configs.

Reference:
  * ``photon-api/.../optimization/RegularizationContext.scala:38-147`` (alpha = 1 for L1, 0 for L2/NONE, param
    (default 0.5) for ELASTIC_NET; L1 weight = alpha*lambda, L2 weight = (1-alpha)*lambda)
  * ``OptimizerConfig.scala:28-47``, ``OptimizerType.scala``, ``OptimizerFactory.scala:38-80``
  * ``game/CoordinateOptimizationConfiguration.scala:22-70`` (FE/RE optimisation configs)
"""
from __future__ import annotations

import enum
import math
from dataclasses import dataclass, field, asdict
from typing import Dict, Optional, Tuple

from ..normalization.context import NormalizationContext
from .lbfgs import LBFGS, OWLQN
from .tron import TRON


class RegularizationType(str, enum.Enum):
    L1 = "L1"
    L2 = "L2"
    ELASTIC_NET = "ELASTIC_NET"
    NONE = "NONE"

    @classmethod
    def parse(cls, s):
        if isinstance(s, RegularizationType):
            return s
        return cls[str(s).strip().upper()]


class OptimizerType(str, enum.Enum):
    LBFGS = "LBFGS"
    TRON = "TRON"

    @classmethod
    def parse(cls, s):
        if isinstance(s, OptimizerType):
            return s
        return cls[str(s).strip().upper()]


@dataclass(frozen=True)
class RegularizationContext:
    regularization_type: RegularizationType = RegularizationType.NONE
    elastic_net_param: Optional[float] = None

    def __post_init__(self):
        rt = RegularizationType.parse(self.regularization_type)
        object.__setattr__(self, "regularization_type", rt)
        if rt != RegularizationType.ELASTIC_NET and self.elastic_net_param is not None:
            raise ValueError("Elastic net parameter can be specified only for elastic net regularization")
        if rt == RegularizationType.ELASTIC_NET and self.elastic_net_param is not None:
            if not (0.0 < self.elastic_net_param <= 1.0):
                raise ValueError(f"Elastic net alpha ({self.elastic_net_param}) is not in interval (0,1].")

    @property
    def alpha(self) -> float:
        rt = self.regularization_type
        if rt == RegularizationType.ELASTIC_NET:
            return 0.5 if self.elastic_net_param is None else float(self.elastic_net_param)
        return 1.0 if rt == RegularizationType.L1 else 0.0

    def l1_weight(self, lam: float) -> float:
        return self.alpha * lam

    def l2_weight(self, lam: float) -> float:
        return (1.0 - self.alpha) * lam

    def to_json(self) -> dict:
        return {"regularizationType": self.regularization_type.value, "elasticNetParam": self.elastic_net_param}


NO_REGULARIZATION = RegularizationContext(RegularizationType.NONE)
L1_REGULARIZATION = RegularizationContext(RegularizationType.L1)
L2_REGULARIZATION = RegularizationContext(RegularizationType.L2)


def elastic_net(alpha: float) -> RegularizationContext:
    return RegularizationContext(RegularizationType.ELASTIC_NET, alpha)


@dataclass
class OptimizerConfig:
    optimizer_type: OptimizerType = OptimizerType.LBFGS
    maximum_iterations: int = 100
    tolerance: float = 1e-7
    constraint_map: Optional[Dict[int, Tuple[float, float]]] = None

    def __post_init__(self):
        self.optimizer_type = OptimizerType.parse(self.optimizer_type)
        if self.maximum_iterations <= 0:
            raise ValueError(f"Less than 1 specified for maximumIterations (specified: {self.maximum_iterations})")
        if self.tolerance < 0:
            raise ValueError(f"Specified negative tolerance for optimizer: {self.tolerance}")

    def to_json(self) -> dict:
        return {"optimizerType": self.optimizer_type.value, "maximumIterations": self.maximum_iterations,
                "tolerance": self.tolerance}


def build_optimizer(config: OptimizerConfig, normalization: Optional[NormalizationContext],
                    reg: RegularizationContext, reg_weight: float = 0.0, track_state: bool = True):
    """OptimizerFactory.build: LBFGS+{L1,EN} -> OWLQN, LBFGS+{L2,NONE} -> LBFGS, TRON+{L2,NONE} -> TRON."""
    ot, rt = config.optimizer_type, reg.regularization_type
    if ot == OptimizerType.LBFGS and rt in (RegularizationType.L1, RegularizationType.ELASTIC_NET):
        return OWLQN(reg.l1_weight(reg_weight), normalization, tolerance=config.tolerance,
                     max_iterations=config.maximum_iterations, constraints=config.constraint_map,
                     track_state=track_state)
    if ot == OptimizerType.LBFGS:
        return LBFGS(normalization, tolerance=config.tolerance, max_iterations=config.maximum_iterations,
                     constraints=config.constraint_map, track_state=track_state)
    if ot == OptimizerType.TRON and rt in (RegularizationType.L2, RegularizationType.NONE):
        return TRON(normalization, tolerance=config.tolerance, max_iterations=config.maximum_iterations,
                    constraints=config.constraint_map, track_state=track_state)
    if ot == OptimizerType.TRON:
        raise ValueError("TRON optimizer incompatible with L1 regularization")
    raise ValueError(f"Incompatible optimizer selected: {ot}")


@dataclass
class GLMOptimizationConfiguration:
    """Per-coordinate optimisation config (FixedEffect/RandomEffectOptimizationConfiguration)."""

    optimizer_config: OptimizerConfig = field(default_factory=OptimizerConfig)
    regularization_context: RegularizationContext = NO_REGULARIZATION
    regularization_weight: float = 0.0
    down_sampling_rate: float = 1.0

    def __post_init__(self):
        if not (0.0 < self.down_sampling_rate <= 1.0):
            raise ValueError(f"Unexpected downSamplingRate: {self.down_sampling_rate}")
        if self.regularization_weight < 0:
            raise ValueError("Negative regularization weight")

    def with_reg_weight(self, w: float) -> "GLMOptimizationConfiguration":
        return GLMOptimizationConfiguration(self.optimizer_config, self.regularization_context, w,
                                            self.down_sampling_rate)

    def to_json(self) -> dict:
        return {
            "optimizerConfig": self.optimizer_config.to_json(),
            "regularizationContext": self.regularization_context.to_json(),
            "regularizationWeight": self.regularization_weight,
            "downSamplingRate": self.down_sampling_rate,
        }

    @staticmethod
    def from_json(d: dict) -> "GLMOptimizationConfiguration":
        oc = d.get("optimizerConfig", {})
        rc = d.get("regularizationContext", {})
        return GLMOptimizationConfiguration(
            OptimizerConfig(oc.get("optimizerType", "LBFGS"), int(oc.get("maximumIterations", 100)),
                            float(oc.get("tolerance", 1e-7))),
            RegularizationContext(rc.get("regularizationType", "NONE"), rc.get("elasticNetParam")),
            float(d.get("regularizationWeight", 0.0)),
            float(d.get("downSamplingRate", 1.0)),
        )


# aliases matching the reference names
FixedEffectOptimizationConfiguration = GLMOptimizationConfiguration
RandomEffectOptimizationConfiguration = GLMOptimizationConfiguration
