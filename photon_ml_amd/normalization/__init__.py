from .context import NormalizationContext, NormalizationType, no_normalization

__all__ = ["NormalizationContext", "NormalizationType", "no_normalization"]
