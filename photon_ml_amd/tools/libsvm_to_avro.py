"""Convert LibSVM text to ``TrainingExampleAvro`` files.

Reference: ``dev-scripts/libsvm_text_to_trainingexample_avro.py`` (Python 2 + avro-python): feature name = the
LibSVM index, term = "", label as given (optionally binarised ``label > 0 -> 1``). Here the native OCF writer is
used and the output can be split into several part files.

Usage: ``python -m photon_ml_amd.tools.libsvm_to_avro input.txt out_dir [--records-per-file N] [--binarize]``
"""
from __future__ import annotations

import argparse
import os
import sys

from ..io.avro import TRAINING_EXAMPLE, write_records


def convert(src: str, out_dir: str, records_per_file: int = 1_000_000, binarize: bool = False,
            codec: str = "deflate") -> int:
    os.makedirs(out_dir, exist_ok=True)
    recs, part, n = [], 0, 0

    def flush():
        nonlocal recs, part
        if recs:
            write_records(os.path.join(out_dir, f"part-{part:05d}.avro"), TRAINING_EXAMPLE, recs, codec=codec)
            part += 1
            recs = []

    with open(src) as f:
        for line in f:
            ts = line.split()
            if not ts:
                continue
            y = float(ts[0])
            if binarize:
                y = 1.0 if y > 0 else 0.0
            feats = []
            for t in ts[1:]:
                k, v = t.split(":")
                feats.append({"name": k, "term": "", "value": float(v)})
            recs.append({"uid": str(n), "label": y, "features": feats, "metadataMap": None, "weight": None,
                         "offset": None})
            n += 1
            if len(recs) >= records_per_file:
                flush()
    flush()
    return n


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("input")
    ap.add_argument("output_dir")
    ap.add_argument("--records-per-file", type=int, default=1_000_000)
    ap.add_argument("--binarize", action="store_true", help="map label > 0 to 1 and everything else to 0")
    ap.add_argument("--codec", default="deflate", choices=["null", "deflate", "snappy"])
    a = ap.parse_args(argv)
    n = convert(a.input, a.output_dir, a.records_per_file, a.binarize, a.codec)
    print(f"wrote {n} records to {a.output_dir}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
