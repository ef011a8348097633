#!/usr/bin/env python3
"""Kernel microbenchmark: per-pass times of the forward (CSR + loss) and transpose (chunked CSC) kernels on the
benchmark data layout, reported as effective stream bandwidth (index + value bytes / time)."""
import argparse
import json
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from photon_ml_amd.data.synthetic import generate_device_shard  # noqa: E402
from photon_ml_amd.function.losses import LOGISTIC  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=8_000_000)
    ap.add_argument("--features", type=int, default=1_000_000)
    ap.add_argument("--nnz", type=int, default=100)
    ap.add_argument("--chunk-rows", type=int, nargs="+", default=[1 << 20])
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--layout", default="auto")
    ap.add_argument("--tl-configs", default="", help="semicolon list of tl_waves,tl_waves_t,tl_pipe (in-process A/B)")
    ap.add_argument("--ablate", type=int, nargs="+", default=[0])
    ap.add_argument("--configs", default="0,1,8192", help="semicolon list of fwd_strided,t_strided,hot_n")
    ap.add_argument("--il", type=int, nargs="+", default=[1], help="tiled stream order(s): 1 lane-interleaved, 0 plain")
    ap.add_argument("--narrow", type=int, nargs="+", default=[1], help="narrow rounds (16-bit packs) off/on")
    args = ap.parse_args()
    res = []
    from photon_ml_amd.ops.native import glm_lib, configure
    lib = glm_lib()
    configs = [tuple(int(v) for v in c.split(",")) for c in args.configs.split(";")]
    if args.tl_configs:
        configs = [("tl",) + tuple(int(v) for v in c.split(",")) for c in args.tl_configs.split(";")]
    cache = {}
    from photon_ml_amd.ops import tiled
    for cr, il, nar, abl, cfg in [(c, i, n, a, g) for c in args.chunk_rows for i in args.il for n in args.narrow
                                  for a in args.ablate for g in configs]:
        lib.pml_set_ablate(0)
        if (cr, il, nar) not in cache:
            cache.clear()
            torch.cuda.empty_cache()
            tiled.INTERLEAVE = il
            tiled.NARROW = nar
            cache[(cr, il, nar)] = generate_device_shard(args.rows, args.features, args.nnz, "cuda", args.precision,
                                                         chunk_rows=cr, layout=args.layout)
        data, w = cache[(cr, il, nar)]
        lib.pml_set_ablate(abl)
        if cfg[0] == "tl":
            configure(tl_waves=cfg[1], tl_waves_t=cfg[2], tl_pipe=cfg[3],
                      tl_multi=cfg[4] if len(cfg) > 4 else 1, tl_pipe_t=cfg[5] if len(cfg) > 5 else cfg[3],
                      tl_deep=cfg[6] if len(cfg) > 6 else 0, tl_deep_t=cfg[7] if len(cfg) > 7 else 0)
        else:
            configure(fwd_strided=cfg[0], t_strided=cfg[1], hot_n=cfg[2])
        x = (w * 0.1).float()
        bytes_per = sum(c.nnz for c in data.csr) * (4 + data.csr[0].val.element_size())
        G = torch.zeros(args.features, dtype=torch.float64, device="cuda")
        nch = len(data.csr)
        # warmup
        data.fwd_all(x, 1, LOGISTIC.loss_id, 0.0, data.coef, None)
        data.t_all(data.coef, G)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        tf, tt = [], []
        for _ in range(args.reps):
            ev[0].record()
            data.fwd_all(x, 1, LOGISTIC.loss_id, 0.0, data.coef, None)
            ev[1].record()
            data.t_all(data.coef, G)
            ev[2].record()
            torch.cuda.synchronize()
            tf.append(ev[0].elapsed_time(ev[1]))
            tt.append(ev[1].elapsed_time(ev[2]))
        t0 = time.perf_counter()
        for _ in range(args.reps):
            data.value_grad_packed(LOGISTIC, w * 0.1, 0.0)
        torch.cuda.synchronize()
        tp = (time.perf_counter() - t0) / args.reps * 1e3
        r = {"cfg": cfg, "il": il, "narrow": nar, "ablate": abl,
             "fwd_stream_GB": sum(c.nbytes() for c in data.csr) / 1e9,
             "t_stream_GB": sum(c.nbytes() for c in data.csc) / 1e9,
             "narrow_frac_fwd": 256 * sum(getattr(c, "n_narrow_rounds", 0) for c in data.csr) / max(1, sum(c.nnz for c in data.csr)),
             "narrow_frac_t": 256 * sum(getattr(c, "n_narrow_rounds", 0) for c in data.csc) / max(1, sum(c.nnz for c in data.csc)), "chunk_rows": cr, "rows": args.rows, "fwd_ms": min(tf), "t_ms": min(tt), "pass_ms": tp,
             "fwd_GBps": bytes_per / min(tf) / 1e6, "t_GBps": bytes_per / min(tt) / 1e6,
             "stream_GB": bytes_per / 1e9, "nblk_fwd": sum(c.nblk for c in data.csr),
             "nblk_t": sum(getattr(c, "nblk", getattr(c, "nitems", 0)) for c in data.csc),
             "nlong_t": sum(getattr(c, "nlong", 0) for c in data.csc), "layout": data.layout}
        print(json.dumps(r), flush=True)
        res.append(r)


if __name__ == "__main__":
    main()
