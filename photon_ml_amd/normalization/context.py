"""Affine per-feature normalisation ``x' = (x - shift) * factor`` folded into the coefficients.

Reference: ``photon-lib/.../normalization/NormalizationContext.scala:39-176`` and
``NormalizationType.scala:20-42``. The transform is never applied to the data (that would destroy sparsity);
instead the objective works on ``w_eff = w * factor`` and a scalar margin shift ``-w_eff . shift``
(``ValueAndGradientAggregator.scala:35-118``).
"""
from __future__ import annotations

import enum
from dataclasses import dataclass
from typing import Optional

import torch


class NormalizationType(str, enum.Enum):
    NONE = "NONE"
    SCALE_WITH_MAX_MAGNITUDE = "SCALE_WITH_MAX_MAGNITUDE"
    SCALE_WITH_STANDARD_DEVIATION = "SCALE_WITH_STANDARD_DEVIATION"
    STANDARDIZATION = "STANDARDIZATION"

    @classmethod
    def parse(cls, s) -> "NormalizationType":
        if isinstance(s, NormalizationType):
            return s
        return cls[str(s).strip().upper()]


@dataclass
class NormalizationContext:
    factors: Optional[torch.Tensor] = None  # fp64 [D]
    shifts: Optional[torch.Tensor] = None  # fp64 [D]
    intercept_id: Optional[int] = None

    def __post_init__(self):
        if self.shifts is not None and self.intercept_id is None:
            raise ValueError("Shift without intercept is illegal.")
        if self.factors is not None and self.shifts is not None and self.factors.numel() != self.shifts.numel():
            raise ValueError("Factors and shifts vectors should have the same size")
        if self.factors is not None and self.intercept_id is not None:
            if float(self.factors[self.intercept_id]) != 1.0:
                raise ValueError("The intercept should not be transformed (factor != 1)")
        if self.shifts is not None and float(self.shifts[self.intercept_id]) != 0.0:
            raise ValueError("The intercept should not be transformed (shift != 0)")

    @property
    def is_identity(self) -> bool:
        return self.factors is None and self.shifts is None

    def to(self, device) -> "NormalizationContext":
        return NormalizationContext(
            None if self.factors is None else self.factors.to(device),
            None if self.shifts is None else self.shifts.to(device),
            self.intercept_id,
        )

    # --- coefficient-space conversions (NormalizationContext.scala:64-111) ---
    def model_to_original_space(self, w: torch.Tensor) -> torch.Tensor:
        if self.factors is None and self.shifts is None:
            return w              # identity: the same tensor (the optimizers never write their iterates in place)
        out = w * self.factors.to(w) if self.factors is not None else w.clone()
        if self.shifts is not None:
            out[self.intercept_id] -= torch.dot(out, self.shifts.to(out))
        return out

    def model_to_transformed_space(self, w: torch.Tensor) -> torch.Tensor:
        if self.factors is None and self.shifts is None:
            return w              # identity (see model_to_original_space): cached margins recognise the tensor
        out = w.clone()
        if self.shifts is not None:
            out[self.intercept_id] += torch.dot(out, self.shifts.to(out))
        if self.factors is not None:
            out = out / self.factors.to(out)
        return out

    # --- effective coefficients used by the kernels ---
    def effective(self, w: torch.Tensor):
        """Return (w_eff, margin_shift) for coefficients ``w`` in transformed space."""
        w_eff = w * self.factors.to(w) if self.factors is not None else w
        shift = -float(torch.dot(w_eff, self.shifts.to(w_eff))) if self.shifts is not None else 0.0
        return w_eff, shift

    def finalize_vector(self, vec_sum: torch.Tensor, prefactor: float) -> torch.Tensor:
        """``g_j = f_j (vecsum_j - s_j * prefactor)`` (ValueAndGradientAggregator.getVector)."""
        out = vec_sum
        if self.shifts is not None:
            out = out - self.shifts.to(out) * prefactor
        if self.factors is not None:
            out = out * self.factors.to(out)
        return out

    @staticmethod
    def build(norm_type, summary, intercept_id: Optional[int]) -> "NormalizationContext":
        """Create from a :class:`BasicStatisticalSummary` (NormalizationContext.scala:124-162)."""
        norm_type = NormalizationType.parse(norm_type)
        if norm_type == NormalizationType.NONE:
            return NormalizationContext(None, None, intercept_id)
        if norm_type == NormalizationType.SCALE_WITH_MAX_MAGNITUDE:
            mag = torch.maximum(summary.max.abs(), summary.min.abs())
            f = torch.where(mag == 0, torch.ones_like(mag), 1.0 / mag)
            return NormalizationContext(f.double(), None, intercept_id)
        std = summary.variance.double().sqrt()
        f = torch.where(std == 0, torch.ones_like(std), 1.0 / std)
        if norm_type == NormalizationType.SCALE_WITH_STANDARD_DEVIATION:
            return NormalizationContext(f, None, intercept_id)
        if norm_type == NormalizationType.STANDARDIZATION:
            if intercept_id is None:
                raise ValueError("STANDARDIZATION requires an intercept")
            s = summary.mean.double().clone()
            s[intercept_id] = 0.0
            f = f.clone()
            f[intercept_id] = 1.0
            return NormalizationContext(f, s, intercept_id)
        raise ValueError(f"NormalizationType {norm_type} not recognized.")


def no_normalization() -> NormalizationContext:
    return NormalizationContext(None, None, None)
