from .optimizer import (ConvergenceReason, OptimizationStatesTracker, Optimizer, OptimizerState,
                        project_box)
from .lbfgs import LBFGS, OWLQN
from .tron import TRON
from .config import (GLMOptimizationConfiguration, OptimizerConfig, OptimizerType, RegularizationContext,
                     RegularizationType, build_optimizer, elastic_net, L1_REGULARIZATION, L2_REGULARIZATION,
                     NO_REGULARIZATION)

__all__ = [
    "ConvergenceReason", "OptimizationStatesTracker", "Optimizer", "OptimizerState", "project_box", "LBFGS",
    "OWLQN", "TRON", "GLMOptimizationConfiguration", "OptimizerConfig", "OptimizerType",
    "RegularizationContext", "RegularizationType", "build_optimizer", "elastic_net", "L1_REGULARIZATION",
    "L2_REGULARIZATION", "NO_REGULARIZATION",
]
