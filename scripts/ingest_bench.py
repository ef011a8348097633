"""Avro -> shard ingest benchmark (SURVEY §2.4 AvroDataReader): synthetic TrainingExample OCF files written
natively (``gen_training_examples``: Zipf-like names, ``--nnz`` features per record, userId tags), then timed
stages: decode (C++ columnar reader, files in parallel), index map + shard assembly (C++ ``assemble_shard``,
row ranges in parallel), and — on a GPU — the device tiled-layout build of the fixed-effect shard. Reports
non-zeros per second per stage and end to end, and the peak RSS.

usage: python scripts/ingest_bench.py --records 10000000 --nnz 100 --files 32 [--dir /tmp/ingest] [--device cuda]
"""
import argparse
import json
import os
import resource
import sys
import time
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=2_000_000)
    ap.add_argument("--nnz", type=int, default=100)
    ap.add_argument("--vocab", type=int, default=1_000_000)
    ap.add_argument("--entities", type=int, default=100_000)
    ap.add_argument("--files", type=int, default=16)
    ap.add_argument("--dir", default="/tmp/pml_ingest")
    ap.add_argument("--codec", default="deflate")
    ap.add_argument("--device", default="none", help="cuda: also build the device tiled layout (bf16 storage)")
    ap.add_argument("--keep", action="store_true", help="keep the generated files")
    ap.add_argument("--out", default=None, help="JSON record path")
    args = ap.parse_args()
    import threading
    t_start = time.perf_counter()
    done = threading.Event()

    def heartbeat():   # long stages print nothing themselves: a line every 30 s shows the run is alive
        while not done.wait(30.0):
            print(f"  ... {time.perf_counter() - t_start:.0f}s, peak RSS "
                  f"{resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20:.1f} GiB", flush=True)
    threading.Thread(target=heartbeat, daemon=True).start()
    from photon_ml_amd.io.avro import native
    from photon_ml_amd.io.data_reader import AvroDataReader, FeatureShardConfiguration
    os.makedirs(args.dir, exist_ok=True)
    per = [args.records // args.files + (1 if i < args.records % args.files else 0) for i in range(args.files)]
    paths = [os.path.join(args.dir, f"part-{i:05d}.avro") for i in range(args.files)]
    t0 = time.perf_counter()
    if not all(os.path.exists(p) for p in paths):
        with ThreadPoolExecutor(max_workers=os.cpu_count()) as ex:
            list(ex.map(lambda a: native().gen_training_examples(a[0], a[1], args.nnz, args.vocab, args.entities,
                                                                 1000 + a[2], args.codec),
                        [(p, n, i) for i, (p, n) in enumerate(zip(paths, per))]))
    t_gen = time.perf_counter() - t0
    size = sum(os.path.getsize(p) for p in paths)
    print(f"generated {args.records} records x {args.nnz} features in {args.files} files ({size / 2**30:.2f} GiB, "
          f"{args.codec}) in {t_gen:.1f}s", flush=True)
    rd = AvroDataReader()
    t0 = time.perf_counter()
    data, maps = rd.read(args.dir, {"global": FeatureShardConfiguration(["features"], True)}, id_tags=["userId"])
    t_read = time.perf_counter() - t0
    x = data.shard("global")
    nnz = int(x.nnz)
    rec = {"records": data.n_rows, "nnz": nnz, "files": args.files, "file_gib": size / 2**30, "codec": args.codec,
           "threads": os.environ.get("PML_AVRO_THREADS", str(os.cpu_count())), "decode_s": rd.timings["decode"],
           "assemble_s": rd.timings["assemble"], "read_s": t_read, "features": x.shape[1],
           "entities": int(len(set(data.id_tags["userId"][:100000])))}
    if args.device != "none":
        import torch
        from photon_ml_amd.ops.device import DeviceGLMData
        t0 = time.perf_counter()
        dev = DeviceGLMData.from_labeled(data.labeled("global"), args.device, "bf16")
        torch.cuda.synchronize()
        rec["device_layout_s"] = time.perf_counter() - t0
        rec["layout"] = dev.layout
    total = sum(v for k, v in rec.items() if k in ("read_s", "device_layout_s"))
    rec.update(total_s=total, nnz_per_s=nnz / total, decode_nnz_per_s=nnz / rec["decode_s"],
               peak_rss_gib=resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20)
    print(json.dumps(rec), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rec, f, indent=1)
    done.set()
    if not args.keep:
        for p in paths:
            os.remove(p)


if __name__ == "__main__":
    main()
