#!/usr/bin/env python3
"""GAME benchmark: fixed + random effect coordinate descent iterations per second (BASELINE.json's second
metric, "GAME coord-descent iters/sec"; config 5 = fixed + per-entity random effects sharded across the GPUs).

Weak scaling: every rank generates ``--entities-per-gpu`` entities x ``--rows-per-entity`` rows (synthetic,
``photon_ml_amd.data.synthetic.generate_game_bench_data``): a ``global`` fixed-effect shard (``--fe-dim``
Zipf features, ``--fe-nnz`` per row + intercept) and an ``entity`` random-effect shard (``--re-dim`` private
features per entity, ``--re-nnz`` per row + intercept). Under torchrun the fixed effect is row-data-parallel (one
packed RCCL all-reduce per evaluation) and the random effect is entity-sharded (all-to-all residual routing);
random-effect solves run as ONE block-diagonal TRON over all owned entities on the GLM HIP kernels.

One STEP = one full coordinate-descent sweep: fixed-effect L-BFGS (``--fe-iters`` iterations) on offsets =
random-effect scores, then the batched per-entity TRON (``--re-iters`` iterations) on offsets = fixed-effect
scores, both rescored, plus the training-loss evaluation. Nothing is skipped inside the timed region.

``--config game5`` = BASELINE.json config 5 at its per-GPU shape: 10M entities x 1k coefficients each over 8
GPUs -> 1.25M entities per GPU, 20 rows x 50 features per entity covering each entity's 1000-feature pool exactly
(+ intercept: 1001 coefficients per entity), integer entity ids, 1M-feature fixed effect.

``--config game5pl`` = the same with power-law entity sizes (see ``generate_game_bench_data(sizes="powerlaw")``).

Usage: python bench_game.py [--gpus N --steps K --warmup W] [--config small|game5|game5pl]; for N > 1 launch with
torch.distributed.run, or let the script start that launcher itself as a child process.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def log(msg):
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench_game {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


PRESETS = {
    "small": dict(entities_per_gpu=200_000, rows_per_entity=50, re_dim=100, re_nnz=10, fe_dim=1_000_000, fe_nnz=30,
                  pool="random", int_ids=0),
    "game5": dict(entities_per_gpu=1_250_000, rows_per_entity=20, re_dim=1000, re_nnz=50, fe_dim=1_000_000,
                  fe_nnz=30, pool="exact", int_ids=1),
    # config 5 with power-law entity sizes (mean 20 rows, Pareto 1.3 tail up to 20k rows): row-space solves for
    # the small entities, the primal block-diagonal solve for the large ones (n_e > 64 or n_e > d_e)
    "game5pl": dict(entities_per_gpu=1_250_000, rows_per_entity=20, re_dim=1000, re_nnz=50, fe_dim=1_000_000,
                    fe_nnz=30, pool="random", int_ids=1, sizes="powerlaw"),
    # game5pl plus a heavy tail: four entities of 45K rows (register-resident workgroup clusters of ~118 members)
    # and three of 150K .. 1M rows (beyond one resident launch: the block-diagonal pass path on its own stream)
    "game5heavy": dict(entities_per_gpu=1_250_000, rows_per_entity=20, re_dim=1000, re_nnz=50, fe_dim=1_000_000,
                       fe_nnz=30, pool="random", int_ids=1, sizes="powerlaw",
                       heavy_rows=(45_000, 45_000, 45_000, 45_000, 150_000, 400_000, 1_000_000)),
    # tall-narrow per-entity models (e.g. per-user models over a few dozen user features, GLMix-style): 250K
    # entities x 100 rows x 31 coefficients (30-feature pools + intercept) — every entity has more rows than
    # coefficients, so each is solved with its exact Hessian on the matrix cores (re_tron_hess_kernel)
    "game5tall": dict(entities_per_gpu=250_000, rows_per_entity=100, re_dim=30, re_nnz=10, fe_dim=1_000_000,
                      fe_nnz=30, pool="random", int_ids=1),
}


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=3,
                    help="untimed sweeps (the first sweeps also grow the caching allocator's pool of model-sized blocks)")
    ap.add_argument("--config", default="small", choices=list(PRESETS))
    ap.add_argument("--entities-per-gpu", type=int)
    ap.add_argument("--rows-per-entity", type=int)
    ap.add_argument("--re-dim", type=int)
    ap.add_argument("--re-nnz", type=int)
    ap.add_argument("--fe-dim", type=int)
    ap.add_argument("--fe-nnz", type=int)
    ap.add_argument("--pool", choices=["random", "exact"])
    ap.add_argument("--int-ids", type=int)
    ap.add_argument("--sizes", choices=["uniform", "powerlaw"])
    ap.add_argument("--heavy-rows", type=lambda v: tuple(int(x) for x in v.split(",") if x),
                    help="comma-separated row counts of extra heavy entities (replacing the first entities' sizes)")
    ap.add_argument("--fe-iters", type=int, default=10)
    ap.add_argument("--re-iters", type=int, default=10)
    ap.add_argument("--label-bias", type=float, default=0.0,
                    help="shift of the ground-truth logit (device data): -4 gives ~5 %% positives (click-like data)")
    ap.add_argument("--fe-down-sampling-rate", type=float, default=1.0,
                    help="fixed-effect down-sampling rate (binary-classification sampler: every positive, negatives "
                         "at this rate, re-weighted); < 1 trains each FE update on a row-sampled copy of the shard")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "f32", "f64"],
                    help="storage precision of the fixed-effect features (accumulation and optimizer state are fp64; "
                         "random-effect features are always fp64)")
    ap.add_argument("--host-data", action="store_true",
                    help="generate the synthetic data with host numpy (minutes at config 5) instead of on the device")
    ap.add_argument("--seed", type=int, default=11)
    ap.add_argument("--rehearsal", action="store_true",
                    help="allow more ranks than physical devices (record: rehearsal true, n_gpus = devices)")
    ap.add_argument("--no-placement", action="store_true",
                    help="multi-rank: route the random-effect rows per coordinate instead of placing every row on "
                         "its entity owner at ingest")
    ap.add_argument("--log-level", default="WARNING",
                    help="framework log level (DEBUG shows the per-phase timings of the random-effect update)")
    return ap


def preset_args(config: str, **overrides) -> argparse.Namespace:
    """Parsed defaults of a preset (what ``bench_game.py --config <config>`` uses), with overrides."""
    args = build_parser().parse_args(["--config", config])
    for k, v in PRESETS[config].items():
        if getattr(args, k) is None:
            setattr(args, k, v)
    for k, v in overrides.items():
        setattr(args, k, v)
    return args


def main():
    args = build_parser().parse_args()
    import logging
    logging.basicConfig(stream=sys.stderr, format="[%(asctime)s %(name)s] %(message)s")
    logging.getLogger("photon_ml_amd").setLevel(args.log_level.upper())
    for k, v in PRESETS[args.config].items():
        if getattr(args, k) is None:
            setattr(args, k, v)
    # --gpus N without a launcher: run N ranks under torch.distributed.run as a child (before any GPU call)
    from photon_ml_amd.parallel.launch import relaunch_if_needed
    rc = relaunch_if_needed(args.gpus, __file__, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)

    import numpy as np
    import torch
    from collections import OrderedDict
    from photon_ml_amd.parallel.dist import init_distributed, all_reduce_scalar, barrier, is_dist
    rank, world, local = init_distributed()
    assert world == args.gpus, (world, args.gpus)
    if torch.cuda.is_available():
        local = local % torch.cuda.device_count()  # several ranks may share a GPU in rehearsal runs
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    from photon_ml_amd.parallel.dist import distinct_devices
    n_dev = distinct_devices(dev)
    if n_dev < world and not args.rehearsal:
        log(f"error: {world} ranks on {n_dev} physical device(s): refusing to report them as {world} GPUs "
            f"(pass --rehearsal for a multi-rank rehearsal on fewer devices)")
        sys.exit(2)
    rec = run(args, dev, rank, world)
    rec["n_gpus"], rec["n_ranks"] = n_dev, world
    if args.rehearsal:
        rec["rehearsal"] = True
    if rank == 0:
        print(json.dumps(rec), flush=True)


def make_data(args, dev, rank: int = 0):
    """The preset's synthetic data for this rank (device generator on a GPU); returns (data, seconds)."""
    import torch
    from photon_ml_amd.data.synthetic import generate_game_bench_data, generate_game_bench_data_device
    t0 = time.time()
    gen_kw = dict(seed=args.seed + 1000 * rank, entity_offset=rank * args.entities_per_gpu, pool=args.pool,
                  int_ids=bool(args.int_ids), sizes=args.sizes or "uniform")
    if args.host_data or dev.type != "cuda":
        data = generate_game_bench_data(args.entities_per_gpu, args.rows_per_entity, args.re_dim, args.re_nnz,
                                        args.fe_dim, args.fe_nnz, **gen_kw)
    else:
        data = generate_game_bench_data_device(args.entities_per_gpu, args.rows_per_entity, args.re_dim, args.re_nnz,
                                               args.fe_dim, args.fe_nnz, device=dev, label_bias=args.label_bias,
                                               heavy_rows=args.heavy_rows or (), **gen_kw)
        torch.cuda.empty_cache()
    t_data = time.time() - t0
    log(f"data generated in {t_data:.1f}s ({'host' if args.host_data or dev.type != 'cuda' else 'device'}): "
        f"{data.n_rows} rows/GPU")
    return data, t_data


def run(args, dev, rank: int = 0, world: int = 1, data=None, t_data: float = 0.0) -> dict:
    """Generate the preset's data (unless given), build the coordinates (fixed-effect storage precision
    ``args.precision``), run ``args.warmup`` untimed and ``args.steps`` timed coordinate-descent sweeps; returns the
    JSON record (rank 0's view; max time over ranks) with the per-sweep min / median next to the mean."""
    import numpy as np
    import torch
    from collections import OrderedDict
    from photon_ml_amd.parallel.dist import all_reduce_scalar, barrier, is_dist
    from photon_ml_amd.algorithm.coordinate_descent import CoordinateDescent
    from photon_ml_amd.algorithm.coordinates import (FixedEffectCoordinate, RandomEffectCoordinate,
                                                     ShardedRandomEffectCoordinate)
    from photon_ml_amd.data.random_effect import FixedEffectDataConfiguration, RandomEffectDataConfiguration
    from photon_ml_amd.evaluation.evaluators import build_evaluator
    from photon_ml_amd.optimization.config import (GLMOptimizationConfiguration, OptimizerConfig,
                                                   RegularizationContext)

    if data is None:
        data, t_data = make_data(args, dev, rank)
    t_place = None
    if is_dist() and not args.no_placement:
        # entity-aligned placement at ingest (parallel/placement.py): every row moves once to the owner of its
        # entity, the fixed effect trains on the placed rows, the random-effect coordinate routes nothing per update
        from photon_ml_amd.parallel.placement import place_rows_by_entity
        tp = time.time()
        data = place_rows_by_entity(data, "entityId", dev)
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        t_place = all_reduce_scalar(time.time() - tp, "max")
        log(f"rows placed on their entity owners in {t_place:.1f}s ({data.placement.rows_moved} rows moved)")
    # the process's first kernel launches (code-object loads, rocBLAS handle, stream creation): measured on their own
    # (ops/warmup.py), so neither the build nor the cold sweep absorbs them; 0.0 when an earlier run paid them
    from photon_ml_amd.ops.warmup import runtime_warmup
    t_warm = all_reduce_scalar(runtime_warmup(dev), "max")
    t0 = time.time()
    # as GameEstimator does: the random-effect shard is copied to the device while the GPU builds the fixed-effect
    # layout (host shards only; placed shards are already device-resident)
    if hasattr(data, "prefetch_shard"):
        data.prefetch_shard("entity", dev)
    fe_cfg = GLMOptimizationConfiguration(OptimizerConfig("LBFGS", args.fe_iters, 1e-12),
                                          RegularizationContext("L2"), 1.0, args.fe_down_sampling_rate)
    re_cfg = GLMOptimizationConfiguration(OptimizerConfig("TRON", args.re_iters, 1e-12),
                                          RegularizationContext("L2"), 1.0)
    task = "LOGISTIC_REGRESSION"
    re_cls = ShardedRandomEffectCoordinate if is_dist() else RandomEffectCoordinate
    coords = OrderedDict([
        ("global", FixedEffectCoordinate("global", data, FixedEffectDataConfiguration("global"), fe_cfg, task,
                                         device=dev, precision=args.precision)),
        ("per-entity", re_cls("per-entity", data, RandomEffectDataConfiguration("entityId", "entity"), re_cfg,
                              task, device=dev)),
    ])
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    t_build = time.time() - t0
    log(f"coordinates built in {t_build:.1f}s (fixed effect {args.precision}); RE: "
        f"{coords['per-entity'].dataset.summary()}")
    # entity-sharded build: per-phase routing seconds (max over ranks)
    route_s = {k: round(all_reduce_scalar(v, "max"), 3)
               for k, v in sorted(getattr(coords["per-entity"], "route_times", {}).items())}
    train_eval = build_evaluator("LOGISTIC_LOSS", data.response, data.offsets, data.weights, device=dev)
    sweep_end = []
    n_coords = len(coords)
    # the training loss after every coordinate update is a host float (a synchronisation), so these stamps are
    # device-complete times; one stamp per sweep (after its last coordinate)
    cb = lambda rec: sweep_end.append(time.perf_counter()) if rec["coordinate"] == list(coords)[-1] else None
    cd = CoordinateDescent(coords, train_eval, score_device=dev, event_callback=cb)
    barrier()
    t_cold = time.perf_counter()
    model, _ = cd.run(args.warmup)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    barrier()
    # the COLD first sweep (every model from zero: the random effects run the most TRON iterations; first-use
    # setup included) — what a one-iteration GAME run (the reference default) costs; warm-up sweep 1
    cold_ms = all_reduce_scalar(1000.0 * (sweep_end[0] - t_cold), "max") if sweep_end else None
    cold_coord_ms = {rec["coordinate"]: 1000.0 * rec["seconds"] for rec in cd.history[:n_coords]}
    fe_gd = coords["global"].glm_data
    fe_pass0 = (getattr(fe_gd, "n_fwd", 0), getattr(fe_gd, "n_t", 0))
    sweep_end.clear()
    t1 = time.perf_counter()
    from photon_ml_amd.utils.timing import trace_range
    with trace_range("timed sweeps"):
        model, _ = cd.run(args.steps, model)
        with trace_range("materialize model"):
            for _, m in model:   # the trained model's coefficients are part of the timed work (row-space RE: lazy)
                if hasattr(m, "materialize"):
                    m.materialize()
            if torch.cuda.is_available():
                torch.cuda.synchronize()
    barrier()
    t_end = time.perf_counter()
    elapsed = all_reduce_scalar(t_end - t1, "max")
    stamps = [t1] + sweep_end[-args.steps:]
    sweeps_ms = [1000.0 * (b - a) for a, b in zip(stamps[:-1], stamps[1:])]
    sweeps_ms = [all_reduce_scalar(v, "max") for v in sweeps_ms]
    log(f"fixed effect per sweep: {(getattr(fe_gd, 'n_fwd', 0) - fe_pass0[0]) / args.steps:.1f} forward + "
        f"{(getattr(fe_gd, 'n_t', 0) - fe_pass0[1]) / args.steps:.1f} transpose passes; sweeps (ms): "
        f"{', '.join(f'{v:.1f}' for v in sweeps_ms)}")
    fe_opt = getattr(getattr(coords["global"], "problem", None), "optimizer", None)
    fe_plans = {k: getattr(fe_opt, k) for k in ("plans_used", "plans_rejected", "wasted_spec_passes", "gated_seen",
                                                 "gated_used") if hasattr(fe_opt, k)}
    if fe_plans:
        log(f"fixed-effect L-BFGS plans (whole run): {fe_plans}")
    loss = cd.history[-1].get("training_loss")
    coord_ms = {}
    for rec in cd.history[-2 * args.steps:]:
        coord_ms.setdefault(rec["coordinate"], []).append(1000.0 * rec["seconds"])
    coord_ms = {k: sum(v) / len(v) for k, v in coord_ms.items()}
    re_stats = coords["per-entity"].last_stats
    total_rows = int(all_reduce_scalar(float(data.n_rows)))
    if rank == 0:
        log(f"final training loss {loss:.6e}; RE stats {re_stats}")
        if torch.cuda.is_available():
            ms = torch.cuda.memory_stats()
            log(f"allocator: peak reserved {ms.get('reserved_bytes.all.peak', 0) / 2**30:.1f} GiB, "
                f"alloc retries {ms.get('num_alloc_retries', 0)}, device mallocs {ms.get('segment.all.allocated', 0)}")
        from photon_ml_amd.optimization.batched import tron_stats
        st = tron_stats()
        if st:
            log(f"block-diagonal TRON: {len(st)} CG steps (all sweeps), mean fraction of rows still iterating "
                f"{sum(st) / len(st):.3f}, min {min(st):.3f}")
        from photon_ml_amd.ops.device import MASK_STATS
        if MASK_STATS:
            fb = sum(a for a, _ in MASK_STATS) / len(MASK_STATS)
            ft = sum(b for _, b in MASK_STATS) / len(MASK_STATS)
            log(f"entity-masked passes: {len(MASK_STATS)} table rebuilds, mean kept fraction: forward blocks "
                f"{fb:.3f}, transpose items {ft:.3f}")
        for rec in cd.history[-2 * args.steps:]:
            log(f"  iteration {rec.get('iteration')} coordinate {rec['coordinate']}: {rec['seconds']:.3f}s")
    route_coords = {k: c for k, c in coords.items() if hasattr(c, "routed_bytes")}
    routing = coords["per-entity"].solver_routing() if hasattr(coords["per-entity"], "solver_routing") else {}
    if rank == 0 and routing:
        log(f"RE solver routing: {routing}")
    del cd, model, train_eval
    return {
        "metric": "GAME coord-descent iters/sec (fixed + per-entity random effect)",
        "value": args.steps / elapsed,
        "unit": "CD iterations/sec",
        "n_gpus": world,            # main() replaces it with the distinct-device count
        "n_ranks": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1000.0 * elapsed / args.steps,
        "sweep_ms_min": min(sweeps_ms) if sweeps_ms else None,
        "cold_first_sweep_ms": cold_ms,
        "cold_first_sweep_coordinate_ms": cold_coord_ms,
        "fe_lbfgs_plans": fe_plans,
        "sweep_ms_median": float(np.median(sweeps_ms)) if sweeps_ms else None,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic (Zipf fixed-effect features, per-entity private random-effect features)",
        "config": {"model": "game_logistic_fe_lbfgs_re_tron", "preset": args.config, "global_batch": total_rows,
                   "seq_len": None, "entity_sizes": args.sizes or "uniform",
                   "entities": args.entities_per_gpu * world, "rows_per_entity": args.rows_per_entity,
                   "re_dim": args.re_dim, "fe_dim": args.fe_dim, "fe_iters": args.fe_iters,
                   "re_iters": args.re_iters, "fe_down_sampling_rate": args.fe_down_sampling_rate,
                   "label_bias": args.label_bias, "positive_fraction": float(np.mean(data.response > 0.5)),
                   "parallelism": f"dp{world}+ep{world}"},
        "coordinate_ms": coord_ms,
        "examples_per_sec": total_rows * args.steps / elapsed,
        "data_generation_s": t_data,
        "runtime_warmup_s": t_warm,
        "coordinate_build_s": t_build,
        # what a one-shot (reference-default, one coordinate-descent iteration) run costs after its data is loaded:
        # warm-up + coordinate build + the cold first sweep
        "one_shot_s": t_warm + t_build + (cold_ms or 0.0) / 1000.0,
        **({"route_s": route_s} if route_s else {}),
        **({"placement_s": t_place} if t_place is not None else {}),
        **({"re_solver_routing": routing} if routing else {}),
        "routed_bytes_per_update": {k: int(all_reduce_scalar(float(getattr(c, "routed_bytes", 0)), "max"))
                                    for k, c in route_coords.items()},
    }


if __name__ == "__main__":
    main()
