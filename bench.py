#!/usr/bin/env python3
"""Headline benchmark: logistic-regression L-BFGS on a 1B x 1M sparse dataset (BASELINE.json config
"Logistic regression L-BFGS bf16 ... 1B rows x 1M sparse feats ... 8xMI355X").

Weak scaling: every GPU owns ``--rows-per-gpu`` rows (default 125M -> 1B rows on 8 GPUs) of a 1M-feature
sparse shard with 100 non-zeros per row (99 Zipf-distributed hashed categorical fields + intercept), features
stored in bf16 in HBM, fp32 products with fp64 accumulation, fp64 optimizer state. Synthetic data generated on
device (no datasets are available offline) — see ``photon_ml_amd/data/synthetic.py``.

One STEP = one full L-BFGS iteration of the production optimizer (``photon_ml_amd.optimization.LBFGS``):
two-loop direction + strong-Wolfe line search, where every trial point is a full pass over the local shard
(fused forward + loss over row blocks, transpose over column tiles — the gather-coalesced "tiled" layout of
``ops/csrc/glm_kernels.hip``) followed by ONE RCCL all-reduce
of the packed fp64 [gradient | loss | sum l'] buffer. Nothing is skipped inside the timed region.

value = (total rows over all ranks) x (L-BFGS iterations) / seconds  [examples/sec/node].

Other BASELINE.json configs (``--config``; per-GPU shapes are the 8-GPU configs divided by 8):

* ``lbfgs``  (default, headline): logistic + L2, L-BFGS, 125M rows/GPU x 1M features;
* ``owlqn``: logistic + L1 (OWL-QN), 125M rows/GPU x 10M features (config "1B rows x 10M sparse feats, 8 GPUs");
* ``tron``:  Poisson + L2, TRON (one STEP = one outer trust-region iteration incl. its Hessian-vector CG passes),
  62.5M rows/GPU x 1M features (config "Poisson regression TRON, 500M rows, 8 GPUs").

Usage: python bench.py [--gpus N --steps K --warmup W] [--config lbfgs|owlqn|tron]; for N > 1 either launch with
torch.distributed.run (one rank per GPU) or let bench.py start that launcher itself as a child process.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def log(msg):
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


CONFIGS = {
    "lbfgs": {"rows_per_gpu": 125_000_000, "features": 1_000_000, "task": "LOGISTIC_REGRESSION",
              "model": "logistic_regression_l2_lbfgs", "metric": "examples/sec/node, logistic L-BFGS 1B×1M-sparse"},
    "owlqn": {"rows_per_gpu": 125_000_000, "features": 10_000_000, "task": "LOGISTIC_REGRESSION",
              "model": "logistic_regression_l1_owlqn",
              "metric": "examples/sec/node, logistic OWL-QN (L1) 1B×10M-sparse"},
    "tron": {"rows_per_gpu": 62_500_000, "features": 1_000_000, "task": "POISSON_REGRESSION",
             "model": "poisson_regression_l2_tron", "metric": "examples/sec/node, Poisson TRON 500M×1M-sparse"},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="lbfgs", choices=list(CONFIGS))
    ap.add_argument("--rows-per-gpu", type=int, default=None)
    ap.add_argument("--features", type=int, default=None)
    ap.add_argument("--nnz", type=int, default=100)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "f32", "f64"])
    ap.add_argument("--chunk-rows", type=int, default=1 << 20)
    ap.add_argument("--l2", type=float, default=1.0)
    ap.add_argument("--l1", type=float, default=10.0, help="L1 weight of the owlqn config")
    ap.add_argument("--seed", type=int, default=1234567890)
    ap.add_argument("--optimizer-state", default="replicated", choices=["replicated", "feature-sharded"],
                    help="replicated: one all-reduce of [g|F|S] per evaluation (default); feature-sharded: w, g and "
                         "the L-BFGS history sharded over features (all-gather w + reduce-scatter g per evaluation)")
    ap.add_argument("--layout", default="auto", choices=["auto", "tiled", "segmented"],
                    help="sparse layout: tiled (gather-coalesced, default when representable) or segmented")
    ap.add_argument("--game", default="auto", choices=["auto", "on", "off"],
                    help="after the timed GLM steps, also time BASELINE.json's GAME metric (coordinate-descent sweeps "
                         "of config 5 with power-law entity sizes, bench_game.py --config game5pl; entity-sharded over "
                         "the ranks when N > 1) with bf16 and with fp64 fixed-effect features, reported as extra "
                         "keys; auto = on for the lbfgs config")
    ap.add_argument("--configs-extra", default="auto", choices=["auto", "on", "off"],
                    help="after the headline (and GAME), also time BASELINE.json configs 3 (OWL-QN, 10M features) and "
                         "4 (Poisson TRON) at fp64 feature storage (the reference's precision; rows reduced to what "
                         "fits in HBM, stated in the keys) and bf16, reported as extra keys; auto = on for the lbfgs "
                         "config at its full size on one rank")
    ap.add_argument("--rehearsal", action="store_true",
                    help="allow more ranks than physical devices (several ranks per GPU, or CPU ranks); the record "
                         "then says rehearsal: true, and n_gpus counts devices, not ranks")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    if args.rows_per_gpu is None:
        args.rows_per_gpu = cfg["rows_per_gpu"]
    if args.features is None:
        args.features = cfg["features"]
    # --gpus N without a launcher: run N ranks under torch.distributed.run as a child (before any GPU call)
    from photon_ml_amd.parallel.launch import relaunch_if_needed
    rc = relaunch_if_needed(args.gpus, __file__, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)

    import torch
    from photon_ml_amd.parallel.dist import init_distributed, DistributedGLMData, all_reduce_scalar, barrier, is_dist
    from photon_ml_amd.parallel.dist import distinct_devices
    rank, world, local = init_distributed()
    assert world == args.gpus, (world, args.gpus)
    local = local % max(torch.cuda.device_count(), 1)  # several ranks may share a GPU in rehearsal runs
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    n_dev = distinct_devices(dev)
    if n_dev < world and not args.rehearsal:
        log(f"error: {world} ranks on {n_dev} physical device(s): refusing to report them as {world} GPUs "
            f"(pass --rehearsal for a multi-rank rehearsal on fewer devices)")
        sys.exit(2)

    import gc
    game = None
    # the GAME metric first, in the process state a GAME user has (no 120 GB of another benchmark's buffers just
    # returned to the driver: after the headline's release the GAME build measured 2.1-5.2 s box to box, 2.0-2.2 s
    # in a fresh process); the headline's timed steps come after its own untimed data generation and warm-up
    if args.game == "on" or (args.game == "auto" and args.config == "lbfgs"):
        game = game_extra(dev, rank, world)
        gc.collect()
        torch.cuda.empty_cache()
    res = glm_run(args.config, args.rows_per_gpu, args.features, args.nnz, args.precision, args.steps, args.warmup,
                  dev, rank, world, args)
    elapsed, st, gnorm, passes, kpass = res["elapsed"], res["state"], res["gnorm"], res["passes"], res["kpass"]
    n_rows_local, layout_name, stalled, total_rows = res["n_rows"], res["layout"], res["stalled"], res["total_rows"]
    sharded = args.optimizer_state == "feature-sharded"
    value = total_rows * args.steps / elapsed
    del res
    gc.collect()
    torch.cuda.empty_cache()
    cfgx = None
    full_size = args.rows_per_gpu == cfg["rows_per_gpu"] and args.features == cfg["features"]
    if args.configs_extra == "on" or (args.configs_extra == "auto" and args.config == "lbfgs" and world == 1
                                      and full_size):
        cfgx = configs_extra(dev, rank, world, args)
    if rank == 0:
        log(f"final f={st.loss:.6e} |g|={gnorm:.3e} evals/step={passes / args.steps:.2f} "
            f"optimizer_stalled={stalled}")
        out = {
            "metric": cfg["metric"],
            "value": value,
            "unit": "examples/sec",
            "n_gpus": n_dev,
            "n_ranks": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1000.0 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.precision,
            "data": "synthetic (on-device Zipf hashed-categorical sparse rows, random ground-truth labels)",
            "config": {
                "model": cfg["model"],
                "global_batch": total_rows,
                "seq_len": None,
                "rows_per_gpu": args.rows_per_gpu,
                "features": args.features,
                "nnz_per_row": args.nnz,
                "parallelism": f"dp{world}" + ("+fs" if sharded else ""),
                "optimizer_state": args.optimizer_state,
                "layout": layout_name,
            },
            "evals_per_step": passes / args.steps,
            "forward_passes_per_step": kpass[0] / args.steps,
            "transpose_passes_per_step": kpass[1] / args.steps,
            "optimizer_stalled": stalled,
        }
        from photon_ml_amd.ops.native import check_lds_add_order
        out["lds_add_order"] = check_lds_add_order(dev)     # determinism premise, verified on this device
        if args.rehearsal:
            out["rehearsal"] = True
        if game is not None:
            out.update(game)
        if cfgx is not None:
            out.update(cfgx)
        print(json.dumps(out), flush=True)


# feature-storage bytes per non-zero of a tiled shard (forward + transpose copies, measured: bf16 115.5 GiB for
# 125M x 100) -- sizes the fp64 runs of configs 3 / 4 to the device memory
BYTES_PER_NNZ = {"bf16": 10.5, "f32": 16.5, "f64": 24.5}


def glm_run(config: str, rows: int, features: int, nnz: int, precision: str, steps: int, warmup: int, dev, rank: int,
            world: int, args) -> dict:
    """Generate the shard of ``config`` on the device and time ``steps`` optimizer iterations after ``warmup``
    untimed ones (max over ranks); the shard is freed on return."""
    import torch
    from photon_ml_amd.parallel.dist import DistributedGLMData, all_reduce_scalar, barrier, is_dist
    from photon_ml_amd.data.synthetic import generate_device_shard
    from photon_ml_amd.utils.timing import trace_range
    from photon_ml_amd.function.losses import LOGISTIC, POISSON
    from photon_ml_amd.function.objective import GLMObjective
    from photon_ml_amd.optimization.lbfgs import LBFGS, OWLQN
    from photon_ml_amd.optimization.tron import TRON
    cfg = CONFIGS[config]
    t_gen = time.time()
    last = [time.time()]

    def progress(i, n):
        if time.time() - last[0] > 20 or i == n:
            last[0] = time.time()
            log(f"generated chunk {i}/{n}")

    data, _ = generate_device_shard(rows, features, nnz, dev, precision, seed=args.seed, chunk_rows=args.chunk_rows,
                                    rank=rank, progress=progress, layout=args.layout, task=cfg["task"])
    torch.cuda.synchronize()
    t_data = time.time() - t_gen
    log(f"[{config} {precision}] data ready in {t_data:.1f}s: {data.n_rows} rows/GPU, "
        f"{data.nbytes() / 2**30:.1f} GiB/GPU, layout={data.layout}")
    sharded = args.optimizer_state == "feature-sharded"
    gdata = DistributedGLMData(data) if is_dist() and not sharded else data
    if is_dist() and not sharded:
        log(f"gradient all-reduce: {'overlapped, %d buckets' % gdata.buckets if gdata.overlap else 'one-shot'}")
    # the optimizer runs exactly warmup + steps iterations (tolerance 0: no early stop), so nothing is queued for an
    # iteration that never runs (L-BFGS speculates the next direction and its margin pass during the history push)
    n_iter = warmup + steps
    if config == "owlqn":
        obj = GLMObjective(LOGISTIC, l2_weight=0.0)
        opt = OWLQN(args.l1, tolerance=0.0, max_iterations=n_iter, track_state=False)
    elif config == "tron":
        obj = GLMObjective(POISSON, l2_weight=args.l2)
        opt = TRON(tolerance=0.0, max_iterations=n_iter, track_state=False)
    else:
        obj = GLMObjective(LOGISTIC, l2_weight=args.l2)
        opt = LBFGS(tolerance=0.0, max_iterations=n_iter, track_state=False)
    import contextlib
    space = contextlib.nullcontext()
    w0 = torch.zeros(features, dtype=torch.float64, device=dev)
    if sharded:
        from photon_ml_amd.optimization.vector_space import ShardedSpace, active_space
        from photon_ml_amd.parallel.feature_sharding import FeatureShardLayout, FeatureShardedObjective
        layout = FeatureShardLayout.current(features)
        obj = FeatureShardedObjective(obj, layout)
        w0 = layout.slice(w0).clone()
        space = active_space(ShardedSpace())
    with space:
        opt.start(obj, gdata, w0, skip_zero_tolerance_pass=True)
        for i in range(warmup):
            st = opt.step(obj, gdata)
            log(f"[{config} {precision}] warmup {i + 1}/{warmup}: f={st.loss:.6e}")
        if hasattr(opt, "drop_speculation"):
            # the last warmup step queued the first timed step's direction + margin pass: drop it, so the timed
            # window holds exactly `steps` forward and `steps` transpose passes
            opt.drop_speculation()
        torch.cuda.synchronize()
        barrier()
        passes0 = data.n_passes
        kpass0 = (getattr(data, "n_fwd", 0), getattr(data, "n_t", 0))
        t0 = time.perf_counter()
        with trace_range("bench timed steps"):  # roctx region (PML_TRACE=1) for timed-window profiles
            for i in range(steps):
                st = opt.step(obj, gdata)
            torch.cuda.synchronize()
        barrier()
        elapsed = time.perf_counter() - t0
        gnorm = st.grad_norm()
    elapsed = all_reduce_scalar(elapsed, "max", device=dev)
    kpass = (getattr(data, "n_fwd", 0) - kpass0[0], getattr(data, "n_t", 0) - kpass0[1])
    out = {"elapsed": elapsed, "state": st, "gnorm": gnorm, "passes": data.n_passes - passes0, "kpass": kpass,
           "n_rows": data.n_rows, "layout": data.layout, "stalled": bool(getattr(opt, "_finished", False)),
           "total_rows": int(all_reduce_scalar(data.n_rows, "sum", device=dev)) if is_dist() else data.n_rows,
           "gib": data.nbytes() / 2**30, "data_s": t_data}
    del data, gdata, opt, obj, w0
    return out


def configs_extra(dev, rank: int, world: int, args) -> dict:
    """BASELINE.json configs 3 (logistic OWL-QN, 1B x 10M over 8 GPUs = 125M rows/GPU x 10M features) and 4 (Poisson
    TRON, 500M rows over 8 GPUs = 62.5M rows/GPU), timed in this run at fp64 feature storage -- the reference computes
    in Double -- with the rows reduced to what fits in this device's memory (stated as ``rows_per_gpu`` next to the
    config's ``config_rows_per_gpu``), and at bf16 (the full row count) for context. Keys ``owlqn10m_<dtype>_*`` and
    ``tron_poisson_<dtype>_*``; each carries its own steps / warmup / passes per step. Failures are reported, never
    fatal to the headline line."""
    import gc
    import torch
    out = {}
    runs = (("owlqn", "owlqn10m", "f64", 5, 2), ("owlqn", "owlqn10m", "bf16", 5, 2),
            ("tron", "tron_poisson", "f64", 3, 1), ("tron", "tron_poisson", "bf16", 3, 1))
    for config, key, prec, steps, warmup in runs:
        cfg = CONFIGS[config]
        pre = f"{key}_{prec}"
        try:
            gc.collect()
            torch.cuda.empty_cache()
            free, _ = torch.cuda.mem_get_info(dev)
            fit = int(0.82 * free / (args.nnz * BYTES_PER_NNZ[prec])) // (1 << 20) * (1 << 20)
            rows = min(cfg["rows_per_gpu"], fit)
            r = glm_run(config, rows, cfg["features"], args.nnz, prec, steps, warmup, dev, rank, world, args)
            out[f"{pre}_ms_per_step"] = 1000.0 * r["elapsed"] / steps
            out[f"{pre}_examples_per_sec"] = r["total_rows"] * steps / r["elapsed"]
            out[f"{pre}_config"] = {
                "model": cfg["model"], "metric": cfg["metric"], "dtype": prec, "rows_per_gpu": r["n_rows"],
                "config_rows_per_gpu": cfg["rows_per_gpu"], "rows_reduced_to_fit": r["n_rows"] < cfg["rows_per_gpu"],
                "features": cfg["features"], "nnz_per_row": args.nnz, "steps": steps, "warmup": warmup,
                "evals_per_step": r["passes"] / steps, "forward_passes_per_step": r["kpass"][0] / steps,
                "transpose_passes_per_step": r["kpass"][1] / steps, "shard_gib": round(r["gib"], 1),
                "optimizer_stalled": r["stalled"], "data_generation_s": round(r["data_s"], 1)}
            log(f"[{config} {prec}] {out[f'{pre}_ms_per_step']:.2f} ms/step over {r['n_rows']} rows "
                f"({r['passes'] / steps:.1f} evaluations/step)")
            del r
        except Exception as e:  # pragma: no cover - reported in the record
            out[f"{pre}_error"] = repr(e)[:500]
            log(f"[{config} {prec}] failed: {e!r}"[:400])
        finally:
            gc.collect()
            torch.cuda.empty_cache()
    return out


def game_extra(dev, rank: int, world: int) -> dict:
    """BASELINE.json's second metric (GAME coordinate-descent iterations/sec, config 5) on the power-law entity
    preset, timed inside this run (bench_game.run: data generated on the device, 2 warmup + 3 timed sweeps, the
    trained model materialised inside the timed region; entity-sharded random effects when world > 1; the cold
    first warm-up sweep, every model from zero, is reported next to the warm mean). Timed twice
    on the same data: bf16 fixed-effect feature storage (``game5pl_*``) and fp64, the reference's precision
    (``game5pl_f64_*``). Failures are reported, never fatal to the GLM line."""
    import gc
    import bench_game
    import torch
    out = {}
    try:
        args = bench_game.preset_args("game5pl", steps=3, warmup=2)
        data, t_data = bench_game.make_data(args, dev, rank)
    except Exception as e:  # pragma: no cover - reported in the record
        return {"game5pl_error": repr(e)[:500]}
    for prec, pre in (("bf16", "game5pl"), ("f64", "game5pl_f64")):
        try:
            args.precision = prec
            g = bench_game.run(args, dev, rank, world, data=data, t_data=t_data)
        except Exception as e:  # pragma: no cover - reported in the record
            out[f"{pre}_error"] = repr(e)[:500]
            continue
        finally:
            gc.collect()
            torch.cuda.empty_cache()
        out.update({f"{pre}_runtime_warmup_s": round(g["runtime_warmup_s"], 3),
                    f"{pre}_coordinate_build_s": round(g["coordinate_build_s"], 3),
                    f"{pre}_one_shot_s": round(g["one_shot_s"], 3),
                    f"{pre}_sweeps_per_sec": g["value"], f"{pre}_ms_per_sweep": g["ms_per_step"],
                    f"{pre}_sweep_ms_min": g["sweep_ms_min"], f"{pre}_sweep_ms_median": g["sweep_ms_median"],
                    f"{pre}_coordinate_ms": g["coordinate_ms"],
                    f"{pre}_cold_first_sweep_ms": g.get("cold_first_sweep_ms"),
                    f"{pre}_cold_first_sweep_coordinate_ms": g.get("cold_first_sweep_coordinate_ms")})
        if g.get("route_s"):
            out[f"{pre}_route_s"] = g["route_s"]
        # multi-rank runs: rows placed on their entity owners at ingest, bytes the RE update still routes
        for k in ("placement_s", "routed_bytes_per_update", "re_solver_routing"):
            if g.get(k) is not None and (k != "routed_bytes_per_update" or world > 1):
                out[f"{pre}_{k}"] = g[k]
        if prec == "bf16":
            out["game5pl_config"] = dict(g["config"], fe_dtype=g["dtype"], re_dtype="fp64", steps=g["steps"],
                                         warmup=g["warmup"], data_generation_s=round(g["data_generation_s"], 1),
                                         coordinate_build_s=round(g["coordinate_build_s"], 3))
    return out


if __name__ == "__main__":
    main()
