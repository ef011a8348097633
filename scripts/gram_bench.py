"""Gram-matrix (21 long fp64 vectors) timing: plain GEMM vs the blocked bmm of vector_space._gram_local."""
import sys, os, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from photon_ml_amd.optimization.vector_space import _gram_local
for n in (1_000_000, 10_000_000):
    vs = [torch.randn(n, dtype=torch.float64, device="cuda") for _ in range(21)]
    V = torch.stack(vs)
    for name, fn in (("gemm", lambda: V @ V.T), ("blocked", lambda: _gram_local(vs))):
        fn(); torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        print(f"n={n} {name}: {(time.perf_counter() - t) / 5 * 1e3:.2f} ms", flush=True)
