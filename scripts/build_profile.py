"""cProfile of the config-5 GAME coordinate construction (FE DeviceGLMData + RE dataset build) on the GPU."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

from photon_ml_amd.algorithm.coordinates import FixedEffectCoordinate, RandomEffectCoordinate
from photon_ml_amd.data.random_effect import FixedEffectDataConfiguration, RandomEffectDataConfiguration
from photon_ml_amd.data.synthetic import generate_game_bench_data
from photon_ml_amd.optimization.config import GLMOptimizationConfiguration, OptimizerConfig, RegularizationContext

scale = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
t = time.time()
data = generate_game_bench_data(int(1_250_000 * scale), 20, 1000, 50, 1_000_000, 30, seed=11, pool="exact",
                                int_ids=True)
print(f"data {time.time() - t:.1f}s rows {data.n_rows}", flush=True)
cfg = GLMOptimizationConfiguration(OptimizerConfig("LBFGS", 10, 1e-12), RegularizationContext("L2"), 1.0)
dev = torch.device("cuda")
pr = cProfile.Profile()
for name, mk in (("FE", lambda: FixedEffectCoordinate("global", data, FixedEffectDataConfiguration("global"), cfg,
                                                      "LOGISTIC_REGRESSION", device=dev, precision="bf16")),
                 ("RE", lambda: RandomEffectCoordinate("per-entity", data,
                                                       RandomEffectDataConfiguration("entityId", "entity"), cfg,
                                                       "LOGISTIC_REGRESSION", device=dev))):
    torch.cuda.synchronize()
    t = time.time()
    pr.enable()
    c = mk()
    torch.cuda.synchronize()
    pr.disable()
    print(f"{name} coordinate built in {time.time() - t:.2f}s", flush=True)
    st = pstats.Stats(pr)
    st.sort_stats("cumulative").print_stats(25)
    pr = cProfile.Profile()
