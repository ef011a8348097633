"""Backend selection for GLM row shards: HIP kernels on a GPU, fp64 torch reference on the CPU.

On a machine with a GPU the native path is the only path (``DeviceGLMData`` raises if its library is missing);
``PML_BACKEND=torch`` forces the reference backend (debugging / parity runs).
"""
from __future__ import annotations

import os

import torch

from ..data.matrix import LabeledData
from .reference import TorchGLMData


def default_device() -> torch.device:
    if os.environ.get("PML_BACKEND") == "torch":
        return torch.device("cpu")
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def make_glm_data(data: LabeledData, device=None, precision: str = "f64", chunk_rows: int = 1 << 20, **kw):
    """``kw`` goes to :meth:`DeviceGLMData.from_labeled` (e.g. ``col_windows=True`` for block-diagonal data)."""
    device = torch.device(device) if device is not None else default_device()
    if device.type == "cuda" and os.environ.get("PML_BACKEND") != "torch":
        from .device import DeviceGLMData
        return DeviceGLMData.from_labeled(data, device, precision, chunk_rows, **kw)
    return TorchGLMData(data, device)
