"""Device runtime warm-up: the once-per-process costs of the first kernel launches, paid up front and measured.

HIP loads a module's code object for a device on the first launch of any kernel in it, and rocBLAS creates its
handle on first use. On MI355X these first launches are tens of milliseconds each (measured in the cold first
GAME sweep, ``profiles/oneshot_r6.md``: one torch reduction kernel's first ``hipLaunchKernel`` 68.7 ms, the first
rocBLAS ``ddot`` 16.5 ms, the first prioritised stream creation 16.5 ms). They are properties of the process, not
of the data or of any solve, so drivers run :func:`runtime_warmup` once before building the coordinates and report
its time as its own figure (``runtime_warmup_s``) instead of letting it land inside whichever solve happens to run
first. Nothing here changes results: every warm-up result is discarded.
"""
from __future__ import annotations

import time

import torch

_DONE = set()


def runtime_warmup(device, force: bool = False) -> float:
    """Launch one small instance of every kernel family the GLM / GAME solvers use on ``device`` (our three HIP
    libraries, torch's elementwise / reduction / norm / scan / sort / index kernels, rocBLAS ``dot``) and create the
    solver side streams. Returns the seconds spent (0.0 when already done in this process, or off the GPU)."""
    dev = torch.device(device)
    if dev.type != "cuda":
        return 0.0
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    if key in _DONE and not force:
        return 0.0
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    from .native import batched_gemv, batched_trsv, check_lds_add_order, csr_gather_rows, key_histogram
    x = torch.linspace(0.0, 1.0, 4096, dtype=torch.float64, device=dev)
    i = torch.arange(4096, dtype=torch.int64, device=dev)
    # torch kernel families of the optimizers, the score algebra and the solver setup
    torch.linalg.vector_norm(x)
    torch.dot(x, x)                                                      # rocBLAS handle + ddot
    (x * x).sum()
    torch.where(x > 0.5, x, torch.zeros_like(x)).square().sum()
    torch.isfinite(x).all()
    torch.cumsum(i, 0)
    torch.sort(i.flip(0), stable=True)
    torch.argsort(x.flip(0), stable=True)
    torch.searchsorted(i, i)
    torch.unique(i % 7, sorted=True, return_inverse=True)
    torch.repeat_interleave(i[:8], i[:8] % 3)
    torch.nonzero(i % 5 == 0)
    x[i.flip(0)]
    torch.zeros_like(x).index_copy_(0, i, x)
    torch.zeros(8, dtype=torch.int64, device=dev).scatter_reduce_(0, i % 8, i, reduce="amax")
    torch.segment_reduce(x, "sum", lengths=torch.full((64,), 64, dtype=torch.int64, device=dev))
    x.to(torch.float32).to(torch.bfloat16)
    # our libraries: the first launch loads each module's code object
    check_lds_add_order(dev)                                             # libpml_glm
    key_histogram(i % 13, 13)                                            # libpml_game
    csr_gather_rows(torch.tensor([0, 2], dtype=torch.int64, device=dev), i[:2], x[:2],
                    torch.zeros(1, dtype=torch.int64, device=dev), torch.tensor([0, 4], dtype=torch.int64, device=dev))
    L = torch.eye(65, dtype=torch.float64, device=dev).unsqueeze(0).contiguous()
    batched_trsv(L, torch.ones(1, 65, dtype=torch.float64, device=dev))  # libpml_re (n > 64)
    batched_gemv(L[:, :8, :8].contiguous(), torch.ones(1, 8, dtype=torch.float64, device=dev))
    torch.cuda.Stream(dev, priority=-1)                                  # first prioritised stream
    torch.cuda.Stream(dev, priority=0)
    torch.cuda.synchronize(dev)
    _DONE.add(key)
    return time.perf_counter() - t0
