#!/usr/bin/env python3
"""10M-key PalDB index map: native build / open / batched lookups (io/csrc/index_map.cpp pml_pdb_*).

    python scripts/paldb_bench.py [--keys 10000000] [--partitions 1,8]
"""
import argparse
import os
import shutil
import sys
import tempfile
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np

from photon_ml_amd.io.paldb import PalDBIndexMap, build_paldb_index_map

ap = argparse.ArgumentParser()
ap.add_argument("--keys", type=int, default=10_000_000)
ap.add_argument("--partitions", default="1,8")
a = ap.parse_args()
t = time.time()
keys = [f"feature{i % 5000}\u0001term{i}" for i in range(a.keys)]
print(f"| keys | partitions | build s | open s | get_indices s (all keys) | keys/s | get_feature_names s (all) | store MB |")
print("|---:|---:|---:|---:|---:|---:|---:|---:|")
for P in (int(x) for x in a.partitions.split(",")):
    d = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        t = time.time()
        build_paldb_index_map(keys, d, "s", P)
        tb = time.time() - t
        t = time.time()
        m = PalDBIndexMap(d, "s", P)
        to = time.time() - t
        t = time.time()
        idx = m.get_indices(keys)
        tg = time.time() - t
        t = time.time()
        names = m.get_feature_names(idx)
        tn = time.time() - t
        assert (idx >= 0).all() and len(m) == a.keys + 1 and names[:1000] == keys[:1000] and names[-1] == keys[-1]
        mb = sum(os.path.getsize(os.path.join(d, f)) for f in os.listdir(d)) / 2**20
        print(f"| {a.keys} | {P} | {tb:.2f} | {to:.4f} | {tg:.2f} | {a.keys / tg / 1e6:.1f}M | {tn:.2f} | {mb:.0f} |",
              flush=True)
        del m
    finally:
        shutil.rmtree(d)
