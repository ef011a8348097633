"""Debug helper: row-space TRON kernel variant V at size n on a few problems -- margins (L beta0) and objective at
the solution against torch (checks the matrix-vector product and the group sums of a variant)."""
import sys
import torch
sys.path.insert(0, ".")
from photon_ml_amd.ops.native import require_glm_lib, rs_tron

n = int(sys.argv[1]) if len(sys.argv) > 1 else 40
V = int(sys.argv[2]) if len(sys.argv) > 2 else 8
B = 3
g = torch.Generator(device="cuda").manual_seed(1)
L = torch.tril(torch.randn(B, n, n, dtype=torch.float64, device="cuda", generator=g))
y = (torch.rand(B, n, device="cuda", generator=g) < 0.5).double()
o = torch.zeros(B, n, dtype=torch.float64, device="cuda")
w = torch.ones(B, n, dtype=torch.float64, device="cuda")
b0 = torch.randn(B, n, dtype=torch.float64, device="cuda", generator=g)
lib = require_glm_lib()
lib.pml_rs_set_variant(V)
z = torch.full_like(b0, float("nan"))
beta, f, it, reason = rs_tron(L, y, o, w, b0, 0, 1.0, 1e-7, 10, zout=z)
torch.cuda.synchronize()
ref_z = torch.bmm(L, beta.unsqueeze(-1)).squeeze(-1)
zz = ref_z
ref_f = (torch.nn.functional.softplus(zz) - y * zz).sum(1) + 0.5 * (beta * beta).sum(1)
print("iters", it.tolist(), "reason", reason.tolist())
print("f", f.tolist(), "ref", ref_f.tolist())
print("max |z - Lb|", (z - ref_z).abs().max().item())
bad = ((z - ref_z).abs() > 1e-9).nonzero()
print("bad entries (problem, index):", bad[:40].tolist())
print("z[0]", z[0].tolist())
print("ref[0]", ref_z[0].tolist())
