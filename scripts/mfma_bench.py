"""Timing + fp64 parity of the hand-written MFMA kernels (game_kernels.hip): gemm_nt (the RANDOM projection's
back-map shape: [entities x k] x [D x k]^T). Run under rocprofv3 --pmc with
SQ_INSTS_VALU_MFMA_* counters for the MFMA evidence (profiles/pmc_mfma_kernels.txt)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from photon_ml_amd.ops.native import gemm_nt

g = torch.Generator(device="cuda").manual_seed(0)
for M, N, K in ((20000, 4096, 128), (4096, 4096, 1024)):
    A = torch.randn(M, K, dtype=torch.float64, device="cuda", generator=g)
    B = torch.randn(N, K, dtype=torch.float64, device="cuda", generator=g)
    C = gemm_nt(A, B)
    ref = A @ B.T
    err = float((C - ref).abs().max() / ref.abs().max())
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        gemm_nt(A, B)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / 5 * 1e3
    print(f"gemm_nt {M}x{N}x{K}: {ms:.3f} ms, {2 * M * N * K / ms / 1e9:.1f} TFLOP/s fp64, rel err {err:.1e}", flush=True)
