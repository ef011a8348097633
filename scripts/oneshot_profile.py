#!/usr/bin/env python3
"""Phase table of a one-shot (reference-default, one coordinate-descent iteration) GAME run on the game5pl preset:
data generation, the coordinate build by phase and the cold first sweep by phase, in a FRESH process.

Run with ``PML_SYNC_TIMED=1`` so every ``Timed`` / ``phase`` block is device-complete (the per-phase numbers then
include a device synchronisation each, which the production run does not pay). Prints one markdown table per
precision and writes ``--json``.

    PML_SYNC_TIMED=1 python scripts/oneshot_profile.py --precisions bf16,f64 --json gpurun_out/oneshot.json
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precisions", default="bf16,f64")
    ap.add_argument("--config", default="game5pl")
    ap.add_argument("--json", default=None)
    ap.add_argument("--cprofile", default=None, help="write cProfile stats of the first run's build + sweep here")
    ap.add_argument("--cprofile-sort", default="cumulative")
    a = ap.parse_args()
    logging.basicConfig(stream=sys.stderr, format="[%(asctime)s %(name)s] %(message)s")
    logging.getLogger("photon_ml_amd").setLevel(logging.DEBUG if os.environ.get("PML_ONESHOT_DEBUG") else
                                                logging.WARNING)
    import torch
    import bench_game
    from photon_ml_amd.utils.timing import TIMELINE
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    t0 = time.time()
    args = bench_game.preset_args(a.config, steps=1, warmup=1)
    data, t_data = bench_game.make_data(args, dev, 0)
    out = {"process_start_to_data_s": round(time.time() - t0, 3), "runs": {}}
    for i, prec in enumerate(a.precisions.split(",")):
        TIMELINE.clear()
        args.precision = prec
        prof = None
        if a.cprofile and i == 0:
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        rec = bench_game.run(args, dev, 0, 1, data=data, t_data=t_data)
        if prof is not None:
            prof.disable()
            import pstats
            with open(a.cprofile, "w") as f:
                pstats.Stats(prof, stream=f).sort_stats(a.cprofile_sort).print_stats(80)
        phases = {k: round(1000.0 * sum(v), 2) for k, v in TIMELINE.items()}
        counts = {k: len(v) for k, v in TIMELINE.items()}
        run = {"runtime_warmup_s": round(rec["runtime_warmup_s"], 3), "coordinate_build_s": round(rec["coordinate_build_s"], 3),
               "cold_first_sweep_ms": round(rec["cold_first_sweep_ms"], 2),
               "cold_first_sweep_coordinate_ms": {k: round(v, 2) for k, v in rec["cold_first_sweep_coordinate_ms"].items()},
               "warm_sweep_ms": round(rec["ms_per_step"], 2), "phases_ms": phases, "phase_counts": counts}
        out["runs"][prec] = run
        print(f"\n## {a.config}, fixed-effect features {prec} (run {i + 1} of the process)\n")
        print(f"runtime warm-up {run['runtime_warmup_s']:.3f} s, coordinate build {run['coordinate_build_s']:.3f} s, cold first sweep {run['cold_first_sweep_ms']:.1f} ms "
              f"{run['cold_first_sweep_coordinate_ms']}, warm sweep {run['warm_sweep_ms']:.1f} ms\n")
        print("| phase | calls | ms |\n|---|---:|---:|")
        for k, v in phases.items():
            print(f"| {k} | {counts[k]} | {v:.1f} |")
        sys.stdout.flush()
        torch.cuda.empty_cache()
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
