"""Microbenchmark of the fused per-entity primal TRON on game5pl-like entities: the streaming kernels
(``stream`` = re_tron_csr_kernel, ``lean`` = re_tron_lean_kernel: rows re-read from memory every pass) vs the
register-resident kernel (``res`` = re_tron_res_kernel: rows loaded once into VGPRs, heavy entities split over
workgroup clusters).

Entities: power-law sizes (Pareto 1.3, 65 .. 20000 rows, the entities the row-space batch does not take at config
5), 1000-feature pools + intercept (d_e <= 1001), 50 distinct pool features per row with N(0,1) values, logistic
labels. Times the whole batch, the largest entities alone, and the rest alone (tail vs throughput bound), and
compares the two kernels' models.

usage: python scripts/re_fused_bench.py [n_entities=43000] [kernels, e.g. stream,res]
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from photon_ml_amd.ops.native import re_lib, re_res_params, re_tron_csr, re_tron_res

E = int(sys.argv[1]) if len(sys.argv) > 1 else 43_000
KERNELS = sys.argv[2].split(",") if len(sys.argv) > 2 else ["stream", "res"]
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
DMAX = int(os.environ.get("PML_BENCH_DMAX", "1008"))     # lean launches: widest entity rounded up to 8
QUAD = os.environ.get("PML_BENCH_QUAD", "1") != "0"     # lean kernel on rows padded to whole quads
nip = torch.arange(N + 1, dtype=torch.int64, device=dev) * NNZ
nip_q, lcol_q, val_q = nip, lcol, val
if QUAD:
    from photon_ml_amd.optimization.entity_tron import pad_rows_to_quads
    nip_q, lcol_q, val_q = pad_rows_to_quads(nip, lcol, val)
y = (torch.rand(N, generator=g, device=dev) < 0.4).double()
off = torch.zeros(N, dtype=torch.float64, device=dev)
wt = torch.ones(N, dtype=torch.float64, device=dev)
scr = torch.empty(4 * N, dtype=torch.float64, device=dev)
print(f"{E} entities, {N} rows, {N * NNZ / 1e6:.0f}M non-zeros, max n_e {int(n_e.max())}", flush=True)

order_all = torch.argsort(n_e, descending=True).to(torch.int32)
top = order_all[:64].contiguous()
rest = order_all[64:].contiguous()
cap, _, grid = re_res_params()


def res_tasks(order):
    ents = order.to(torch.int64)
    k = (n_e[ents] + cap - 1) // cap
    key = k * (int(n_e.max()) * NNZ + 1) + n_e[ents] * NNZ
    ents = ents[torch.argsort(key, descending=True, stable=True)]
    k = (n_e[ents] + cap - 1) // cap
    t0 = torch.zeros(ents.numel() + 1, dtype=torch.int64, device=dev)
    torch.cumsum(k, 0, out=t0[1:])
    ncl = int(k[k > 1].sum())
    ws = torch.empty(int(re_lib().pml_re_res_ws_doubles(max(ncl, 1))), dtype=torch.float64, device=dev)
    return ents.to(torch.int32).contiguous(), t0.to(torch.int32).contiguous(), ws, int((k > 1).sum())


def run(kernel, order, reps=3):
    W = torch.zeros(E * d, dtype=torch.float64, device=dev)
    f = torch.empty(E, dtype=torch.float64, device=dev)
    it = torch.empty(E, dtype=torch.int32, device=dev)
    rc = torch.empty(E, dtype=torch.int32, device=dev)
    z = torch.empty(N, dtype=torch.float64, device=dev)
    npass = torch.zeros(E, dtype=torch.int32, device=dev)
    if kernel == "res":
        te, t0, ws, ncl = res_tasks(order)

        def call(np_=None):
            return re_tron_res(te, t0, ws, grid, row_ptr, col_ptr, nip, lcol, val, y, off, wt, W, f, it, rc, z, 0,
                               1.0, 1e-12, 10, 5, 20, npass=np_)
    else:
        def call(np_=None):
            q = kernel == "lean" and QUAD
            re_tron_csr(order, row_ptr, col_ptr, nip_q if q else nip, lcol_q if q else lcol, val_q if q else val, y,
                        off, wt, scr, W, f, it, rc, z, 0, 1.0, 1e-12, 10, 5, 20, DMAX if kernel == "lean" else 1024,
                        npass=np_, lean=kernel == "lean", quad=q)
            return None
    err = call(npass)
    torch.cuda.synchronize()
    assert err is None or int(err.item()) == 0, "cluster wait timed out"
    t = time.perf_counter()
    for _ in range(reps):
        W.zero_()
        call()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / reps * 1e3
    sel = order.to(torch.int64)
    # bytes per row pass: 10 per non-zero (int16 column + fp64 value) + ~16 per row (row pointer, D / y, off, wt)
    gb = float((npass[sel].double() * (n_e[sel] * (NNZ * 10 + 16)).double()).sum()) / 1e9
    return ms, it.clone(), gb, float(npass[sel].double().mean()), W.clone(), z.clone()


models = {}
for kern in KERNELS:
    t_all, it, gb, mp, W, z = run(kern, order_all)
    models[kern] = (W, z, it)
    t_top, _, gb_top, mp_top, _, _ = run(kern, top)
    t_rest, _, gb_rest, _, _, _ = run(kern, rest)
    print(f"{kern}: all {t_all:.2f} ms ({gb:.1f} GB of row passes, {gb / t_all:.2f} TB/s equivalent, mean passes/entity "
          f"{mp:.1f}) | 64 largest alone {t_top:.2f} ms | the rest {t_rest:.2f} ms | mean TRON iterations "
          f"{it.double().mean():.3f}", flush=True)
if len(models) == 2:
    (Wa, za, ia), (Wb, zb, ib) = models.values()
    print(f"max |W diff| {float((Wa - Wb).abs().max()):.3e}, max |z diff| {float((za - zb).abs().max()):.3e}, "
          f"iteration counts equal for {float((ia == ib).double().mean()) * 100:.2f} % of entities", flush=True)
