"""Microbenchmark of the fused row-space TRON kernel variants (config-5 shape: 1.25M problems of 20 x 20)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import time

import torch

from photon_ml_amd.ops.native import require_glm_lib, rs_tron

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1_250_000
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
g = torch.Generator(device="cuda").manual_seed(0)
X = torch.randn(B, n, 3 * n, dtype=torch.float64, device="cuda", generator=g) * 0.3
K = X @ X.transpose(1, 2)
L = torch.linalg.cholesky(K)
del X, K
y = (torch.rand(B, n, device="cuda", generator=g) < 0.5).double()
o = torch.zeros(B, n, dtype=torch.float64, device="cuda")
w = torch.ones(B, n, dtype=torch.float64, device="cuda")
b0 = torch.zeros(B, n, dtype=torch.float64, device="cuda")
lib = require_glm_lib()
res = {}
VARIANTS = [int(v) for v in sys.argv[3].split(",")] if len(sys.argv) > 3 else [2, 3]
for v in VARIANTS + VARIANTS:
    lib.pml_rs_set_variant(v)
    out = rs_tron(L, y, o, w, b0, 0, 1.0, 1e-7, 10)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(3):
        out = rs_tron(L, y, o, w, b0, 0, 1.0, 1e-7, 10)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / 3 * 1e3
    res[v] = out
    print(f"variant {v}: {ms:.2f} ms  mean iters {out[2].double().mean():.3f}", flush=True)
v0 = VARIANTS[0]
for v in VARIANTS[1:]:
    d = (res[v0][0] - res[v][0]).abs().max().item()
    fr = (res[v0][2] != res[v][2]).double().mean().item()
    print(f"variant {v} vs {v0}: max |beta diff| = {d:.3e}; iteration counts differ on {fr:.4%} of problems")
# problem order grouped by iteration count (what optimization/row_space.py passes from the previous solve)
vlast = VARIANTS[-1]
lib.pml_rs_set_variant(vlast)
order = torch.argsort(res[vlast][2], stable=True).to(torch.int32)
for _ in range(2):
    out = rs_tron(L, y, o, w, b0, 0, 1.0, 1e-7, 10, order=order)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(3):
        out = rs_tron(L, y, o, w, b0, 0, 1.0, 1e-7, 10, order=order)
    torch.cuda.synchronize()
    print(f"variant {vlast} ordered by iterations: {(time.perf_counter() - t) / 3 * 1e3:.2f} ms; bitwise equal to "
          f"entity order: {bool(torch.equal(out[0], res[vlast][0]) and torch.equal(out[2], res[vlast][2]))}",
          flush=True)
