"""Microbenchmark of the fused per-entity primal TRON (re_tron_csr_kernel) on game5pl-like entities.

Entities: power-law sizes (Pareto 1.3, 65 .. 20000 rows, the entities the row-space batch does not take at config
5), 1000-feature pools + intercept (d_e <= 1001), 50 distinct pool features per row with N(0,1) values, logistic
labels. Times the whole batch, the largest entities alone, and the rest alone — whether the launch is bound by
its longest entity (one workgroup) or by aggregate throughput.

usage: python scripts/re_fused_bench.py [n_entities=43000] [variant list, e.g. 2,1]
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from photon_ml_amd.ops.native import re_lib, re_tron_csr

E = int(sys.argv[1]) if len(sys.argv) > 1 else 43_000
VARIANTS = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [2]
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(1)
u = torch.rand(E, generator=g, device=dev, dtype=torch.float64)
n_e = torch.clamp(torch.ceil(65.0 * u ** (-1.0 / 1.3)), max=20000).to(torch.int64)
N = int(n_e.sum())
NNZ = 51
d = 1001
row_ptr = torch.zeros(E + 1, dtype=torch.int64, device=dev)
torch.cumsum(n_e, 0, out=row_ptr[1:])
col_ptr = torch.arange(E + 1, dtype=torch.int64, device=dev) * d
# 50 distinct pool features per row: a + k s mod 1000 with s coprime to 1000
strides = torch.tensor([s for s in range(1, 200) if s % 2 and s % 5], device=dev)
a = torch.randint(0, d - 1, (N, 1), generator=g, device=dev)
s_ = strides[torch.randint(0, strides.numel(), (N, 1), generator=g, device=dev)]
cols = (a + torch.arange(NNZ - 1, device=dev)[None, :] * s_) % (d - 1)
cols, _ = torch.sort(cols, dim=1)
lcol = torch.cat([cols, torch.full((N, 1), d - 1, device=dev)], 1).reshape(-1).to(torch.int16)
del cols
val = torch.randn(N * NNZ, generator=g, device=dev, dtype=torch.float64)
val.view(N, NNZ)[:, -1] = 1.0
nip = torch.arange(N + 1, dtype=torch.int64, device=dev) * NNZ
y = (torch.rand(N, generator=g, device=dev) < 0.4).double()
off = torch.zeros(N, dtype=torch.float64, device=dev)
wt = torch.ones(N, dtype=torch.float64, device=dev)
scr = torch.empty(4 * N, dtype=torch.float64, device=dev)
print(f"{E} entities, {N} rows, {N * NNZ / 1e6:.0f}M non-zeros, max n_e {int(n_e.max())}", flush=True)

order_all = torch.argsort(n_e, descending=True).to(torch.int32)
top = order_all[:64].contiguous()
rest = order_all[64:].contiguous()


def run(order, reps=3):
    W = torch.zeros(E * d, dtype=torch.float64, device=dev)
    f = torch.empty(E, dtype=torch.float64, device=dev)
    it = torch.empty(E, dtype=torch.int32, device=dev)
    rc = torch.empty(E, dtype=torch.int32, device=dev)
    z = torch.empty(N, dtype=torch.float64, device=dev)
    npass = torch.zeros(E, dtype=torch.int32, device=dev)
    args = (row_ptr, col_ptr, nip, lcol, val, y, off, wt, scr)
    re_tron_csr(order, *args, W, f, it, rc, z, 0, 1.0, 1e-12, 10, 5, 20, 1024, npass=npass)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        W.zero_()
        re_tron_csr(order, *args, W, f, it, rc, z, 0, 1.0, 1e-12, 10, 5, 20, 1024)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / reps * 1e3
    sel = order.to(torch.int64)
    # bytes per row pass: 10 per non-zero (int16 column + fp64 value) + ~16 per row (row pointer, D / y, off, wt)
    gb = float((npass[sel].double() * (n_e[sel] * (NNZ * 10 + 16)).double()).sum()) / 1e9
    return ms, it, gb, float(npass[sel].double().mean())


lib = re_lib()
for v in VARIANTS:
    lib.pml_re_set_variant(v)
    t_all, it, gb, mp = run(order_all)
    t_top, _, gb_top, mp_top = run(top)
    t_rest, _, gb_rest, _ = run(rest)
    print(f"variant {v}: all {t_all:.2f} ms ({gb:.1f} GB streamed, {gb / t_all:.2f} TB/s, mean passes/entity "
          f"{mp:.1f}) | 64 largest alone {t_top:.2f} ms ({gb_top / t_top:.2f} TB/s, {mp_top:.1f} passes) | "
          f"the rest {t_rest:.2f} ms ({gb_rest / t_rest:.2f} TB/s) | mean TRON iterations {it.double().mean():.2f}",
          flush=True)
