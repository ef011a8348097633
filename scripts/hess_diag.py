"""Diagnostic: fused exact-Hessian RE TRON vs fused sparse-Hv vs pass path on the d_user=40 Poisson test data, at
the test tolerance and at a tight tolerance; prints the worst entity's differences."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch

import photon_ml_amd.optimization.entity_tron as et
from photon_ml_amd.algorithm.coordinates import RandomEffectCoordinate
from photon_ml_amd.data.game_data import generate_game_data
from photon_ml_amd.data.random_effect import RandomEffectDataConfiguration
from photon_ml_amd.optimization.config import GLMOptimizationConfiguration, OptimizerConfig, RegularizationContext

task = sys.argv[1] if len(sys.argv) > 1 else "POISSON_REGRESSION"
d_user = int(sys.argv[2]) if len(sys.argv) > 2 else 40
data, _ = generate_game_data(n_rows=30000, n_users=700, d_user=d_user, seed=26, task=task)
for tol, iters in ((1e-10, 30), (1e-14, 300)):
    res = {}
    for name, fused, hess in (("pass", "0", 64), ("sparse", "1", 0), ("hess", "1", 64)):
        os.environ["PML_RE_FUSED"] = fused
        et.HESS_DMAX = hess
        cfg = GLMOptimizationConfiguration(OptimizerConfig("TRON", iters, tol), RegularizationContext("L2"), 1.0)
        c = RandomEffectCoordinate("u", data, RandomEffectDataConfiguration("userId", "user"), cfg, task,
                                   device="cuda", layout="segmented")
        m1 = c.update_model(c.initialize_model())
        res[name] = (np.asarray(m1.values).copy(), c.last_stats)
    for a, b in (("pass", "sparse"), ("pass", "hess"), ("sparse", "hess")):
        va, vb = res[a][0], res[b][0]
        d = np.abs(va - vb)
        i = int(d.argmax())
        print(f"tol {tol:g} iters {iters}: {a} vs {b}: max abs {d.max():.3e} at {i} (values {va[i]:.10g} {vb[i]:.10g}),"
              f" rel {float((d / np.maximum(np.abs(va), 1e-12)).max()):.3e}, n>1e-8: {int((d > 1e-8).sum())}", flush=True)
    for k, (_, st) in res.items():
        print(f"  {k}: {st}", flush=True)
