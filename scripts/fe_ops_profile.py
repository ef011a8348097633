"""Where the small launches of a GAME fixed-effect update come from: torch.profiler over ONE warm FE coordinate
update of a preset (default game5pl), device kernels and memcpys attributed to the innermost photon_ml_amd source
line on the launching stack. usage: python scripts/fe_ops_profile.py [preset] [out.txt]"""
import collections
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch

import bench_game
from photon_ml_amd.algorithm.coordinate_descent import CoordinateDescent
from photon_ml_amd.algorithm.coordinates import FixedEffectCoordinate, RandomEffectCoordinate
from photon_ml_amd.data.random_effect import FixedEffectDataConfiguration, RandomEffectDataConfiguration
from photon_ml_amd.evaluation.evaluators import build_evaluator
from photon_ml_amd.optimization.config import GLMOptimizationConfiguration, OptimizerConfig, RegularizationContext

preset = sys.argv[1] if len(sys.argv) > 1 else "game5pl"
out = sys.argv[2] if len(sys.argv) > 2 else None
dev = torch.device("cuda")
args = bench_game.preset_args(preset)
data, _ = bench_game.make_data(args, dev)
fe_cfg = GLMOptimizationConfiguration(OptimizerConfig("LBFGS", 10, 1e-12), RegularizationContext("L2"), 1.0)
re_cfg = GLMOptimizationConfiguration(OptimizerConfig("TRON", 10, 1e-12), RegularizationContext("L2"), 1.0)
from collections import OrderedDict
coords = OrderedDict([
    ("global", FixedEffectCoordinate("global", data, FixedEffectDataConfiguration("global"), fe_cfg,
                                     "LOGISTIC_REGRESSION", device=dev, precision="bf16")),
    ("per-entity", RandomEffectCoordinate("per-entity", data, RandomEffectDataConfiguration("entityId", "entity"),
                                          re_cfg, "LOGISTIC_REGRESSION", device=dev)),
])
ev = build_evaluator("LOGISTIC_LOSS", data.response, data.offsets, data.weights, device=dev)
cd = CoordinateDescent(coords, ev, score_device=dev)
model, _ = cd.run(2)
fe = coords["global"]
scores = {cid: c.score(model.get(cid)).to(dev) for cid, c in coords.items()}
partial = scores["per-entity"]
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    fe.update_model(model.get("global"), partial)
    torch.cuda.synchronize()
ops = collections.Counter()
for e in prof.events():
    if not e.name.startswith("aten::") or e.name in ("aten::empty", "aten::empty_strided", "aten::view",
                                                     "aten::as_strided", "aten::resize_", "aten::item"):
        continue
    if getattr(e, "cpu_parent", None) is not None and e.cpu_parent.name.startswith("aten::"):
        continue                                   # count top-level aten calls only
    fr = [f for f in (e.stack or []) if "photon_ml_amd" in f]
    ops[(e.name, fr[0] if fr else "?", fr[1] if len(fr) > 1 else "")] += 1
lines = [f"{n:4d}  {name:28s} {f0}  <- {f1}" for (name, f0, f1), n in ops.most_common(60)]
tab = "\n".join(lines)
cnt = prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=40)
print(tab)
if out:
    open(out, "w").write(tab + "\n\n" + cnt)
