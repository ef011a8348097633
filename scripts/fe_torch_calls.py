"""Which torch calls a warm GAME fixed-effect (and random-effect) coordinate update issues, attributed to the
innermost photon_ml_amd source line (a TorchFunctionMode logger: works where the profiler's Python stacks do not).
usage: python scripts/fe_torch_calls.py [preset] [out.txt]"""
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
from torch.overrides import TorchFunctionMode

import bench_game
from collections import OrderedDict
from photon_ml_amd.algorithm.coordinate_descent import CoordinateDescent
from photon_ml_amd.algorithm.coordinates import FixedEffectCoordinate, RandomEffectCoordinate
from photon_ml_amd.data.random_effect import FixedEffectDataConfiguration, RandomEffectDataConfiguration
from photon_ml_amd.evaluation.evaluators import build_evaluator
from photon_ml_amd.optimization.config import GLMOptimizationConfiguration, OptimizerConfig, RegularizationContext

SKIP = {"__get__", "size", "dim", "numel", "__len__", "is_cuda", "dtype", "device", "shape", "data_ptr",
        "is_contiguous", "__repr__", "__format__", "stride", "element_size", "__bool__", "__index__", "__int__",
        "__float__", "tolist", "item", "__hash__", "__eq__", "storage_offset", "is_floating_point"}


class Calls(TorchFunctionMode):
    def __init__(self):
        super().__init__()
        self.c = collections.Counter()

    def __torch_function__(self, func, types, args=(), kwargs=None):
        name = getattr(func, "__name__", str(func))
        if name not in SKIP:
            fr = [f for f in traceback.extract_stack()[:-1] if "photon_ml_amd" in f.filename]
            where = f"{os.path.relpath(fr[-1].filename)}:{fr[-1].lineno}" if fr else "?"
            self.c[(name, where)] += 1
        return func(*args, **(kwargs or {}))


preset = sys.argv[1] if len(sys.argv) > 1 else "game5pl"
out = sys.argv[2] if len(sys.argv) > 2 else None
dev = torch.device("cuda")
args = bench_game.preset_args(preset)
data, _ = bench_game.make_data(args, dev)
fe_cfg = GLMOptimizationConfiguration(OptimizerConfig("LBFGS", 10, 1e-12), RegularizationContext("L2"), 1.0)
re_cfg = GLMOptimizationConfiguration(OptimizerConfig("TRON", 10, 1e-12), RegularizationContext("L2"), 1.0)
coords = OrderedDict([
    ("global", FixedEffectCoordinate("global", data, FixedEffectDataConfiguration("global"), fe_cfg,
                                     "LOGISTIC_REGRESSION", device=dev, precision="bf16")),
    ("per-entity", RandomEffectCoordinate("per-entity", data, RandomEffectDataConfiguration("entityId", "entity"),
                                          re_cfg, "LOGISTIC_REGRESSION", device=dev)),
])
ev = build_evaluator("LOGISTIC_LOSS", data.response, data.offsets, data.weights, device=dev)
cd = CoordinateDescent(coords, ev, score_device=dev)
model, _ = cd.run(2)
torch.cuda.synchronize()
text = []
log = Calls()
with log:
    model, _ = cd.run(1, model)
torch.cuda.synchronize()
text.append(f"# one coordinate-descent sweep (both coordinates + training loss): {sum(log.c.values())} torch calls")
text += [f"{n:4d}  {name:32s} {where}" for (name, where), n in log.c.most_common(70)]
# the random-effect coordinate update alone (calls made inside RandomEffectCoordinate.update_model)
re_coord = coords["per-entity"]
partial = cd.coordinates["global"].score(model.get("global"))
log = Calls()
with log:
    re_coord.update_model(model.get("per-entity"), partial)
torch.cuda.synchronize()
text.append(f"# random-effect coordinate update alone: {sum(log.c.values())} torch calls")
text += [f"{n:4d}  {name:32s} {where}" for (name, where), n in log.c.most_common(80)]
print("\n".join(text))
if out:
    open(out, "w").write("\n".join(text) + "\n")
