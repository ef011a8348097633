#!/usr/bin/env python3
"""The primary entry point end to end at scale: Avro TrainingExample files -> ``game-training`` (GameTrainingDriver:
read, index, build, ONE coordinate-descent iteration -- the reference default -- of a fixed effect + per-user random
effect, save the model as Avro) on one GPU, with the driver's own phase timers (``Timed`` blocks, device-complete
with ``PML_SYNC_TIMED=1``).

Data: ``gen_training_examples`` (native, ``io/csrc/avro_codec.cpp``): ``--records`` records of ``--nnz`` Zipf-like
features from a ``--vocab``-name vocabulary, ``--entities`` user ids; the same feature bag feeds the fixed-effect
shard and the per-user random-effect shard (+ intercepts), as in Photon's common global + per-user setups.

    python scripts/cli_oneshot.py --records 10000000 --nnz 30 --entities 500000 --dir /tmp/cli_oneshot
"""
import argparse
import json
import os
import shutil
import sys
import time
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=10_000_000)
    ap.add_argument("--nnz", type=int, default=30)
    ap.add_argument("--vocab", type=int, default=1_000_000)
    ap.add_argument("--entities", type=int, default=500_000)
    ap.add_argument("--files", type=int, default=32)
    ap.add_argument("--dir", default="/tmp/pml_cli_oneshot")
    ap.add_argument("--precision", default="f64")
    ap.add_argument("--out", default=None, help="JSON record path")
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args()
    from photon_ml_amd.io.avro import native
    data_dir = os.path.join(a.dir, "train")
    os.makedirs(data_dir, exist_ok=True)
    per = [a.records // a.files + (1 if i < a.records % a.files else 0) for i in range(a.files)]
    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
        list(ex.map(lambda t: native().gen_training_examples(os.path.join(data_dir, f"part-{t[0]:05d}.avro"), t[1],
                                                              a.nnz, a.vocab, a.entities, 500 + t[0], "deflate"),
                    list(enumerate(per))))
    t_gen = time.perf_counter() - t0
    size = sum(os.path.getsize(os.path.join(data_dir, f)) for f in os.listdir(data_dir))
    print(f"generated {a.records} records x {a.nnz} features ({size / 2**30:.2f} GiB) in {t_gen:.1f}s", flush=True)
    from photon_ml_amd.cli import game_training
    from photon_ml_amd.utils.timing import TIMELINE
    out = os.path.join(a.dir, "out")
    args = ["--input-data-directories", data_dir, "--root-output-directory", out,
            "--training-task", "LOGISTIC_REGRESSION",
            "--feature-shard-configurations", "name=global,feature.bags=features",
            "--feature-shard-configurations", "name=user,feature.bags=features,intercept=true",
            "--coordinate-configurations",
            "name=fixed,feature.shard=global,optimizer=LBFGS,max.iter=10,tolerance=1e-7,regularization=L2,reg.weights=1",
            "--coordinate-configurations",
            "name=per-user,feature.shard=user,random.effect.type=userId,optimizer=TRON,max.iter=10,tolerance=1e-7,"
            "regularization=L2,reg.weights=1",
            "--coordinate-update-sequence", "fixed,per-user", "--coordinate-descent-iterations", "1",
            "--output-mode", "BEST", "--device", a.device, "--precision", a.precision]
    t0 = time.perf_counter()
    res = game_training.GameTrainingDriver(game_training.build_parser().parse_args(args)).run()
    total = time.perf_counter() - t0
    phases = {k: round(sum(v), 3) for k, v in TIMELINE.items()}
    model_bytes = sum(os.path.getsize(os.path.join(r, f)) for r, _, fs in os.walk(out) for f in fs)
    rec = {"records": a.records, "nnz_per_record": a.nnz, "entities": a.entities, "vocab": a.vocab,
           "precision": a.precision, "avro_gib": round(size / 2**30, 2), "driver_total_s": round(total, 2),
           "model_mib": round(model_bytes / 2**20, 1), "phases_s": phases}
    print(json.dumps(rec, indent=1), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rec, f, indent=1)
    shutil.rmtree(a.dir, ignore_errors=True)


if __name__ == "__main__":
    main()
