"""Timing of the L-BFGS two-loop Gram kernel (fp64 MFMA, ``gram_kernel``) and the whole vector-free device
two-loop at the headline / GAME size (n = 1M coefficients, 10 history pairs -> 21 vectors).
usage: python scripts/gram_mfma_bench.py"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from photon_ml_amd.ops.native import gram, two_loop_gram

for n in (1_000_000, 10_000_000):
    g = torch.Generator(device="cuda").manual_seed(1)
    vs = [torch.randn(n, dtype=torch.float64, device="cuda", generator=g) for _ in range(21)]
    V = torch.stack(vs)
    err = float(((gram(vs) - V @ V.T).abs().max() / (V @ V.T).abs().max()))
    for name, fn in (("gram (21 vectors)", lambda: gram(vs)),
                     ("two-loop gram (10 pairs)", lambda: two_loop_gram(vs[:10], vs[10:20], vs[20]))):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) / 20 * 1e3
        print(f"n={n} {name}: {ms:.3f} ms ({21 * n * 8 / ms / 1e9:.2f} TB/s of basis reads); max rel err {err:.2e}",
              flush=True)
