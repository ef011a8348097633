"""Evaluation metrics, model / training diagnostics and report rendering (photon-diagnostics)."""
from .evaluation import evaluate, select_best_model  # noqa: F401
