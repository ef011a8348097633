"""Feature-space preparation CLIs: off-heap index maps and name/term feature-bag lists.

Reference:
  * ``photon-client/.../index/FeatureIndexingDriver.scala:40-260`` — scan the input Avro, collect the distinct
    ``name\\u0001term`` keys of each feature shard's bags (+ the intercept when the shard has one), partition them
    and write one PalDB store per (shard, partition) under the output directory.
    Here: one memory-mapped hash-table store per partition built by the native ``io/csrc/index_map.cpp``
    (:func:`photon_ml_amd.io.index_map.build_offheap_index_map`), loaded with ``OffHeapIndexMap``; or, with
    ``--index-format paldb``, PalDB V1 stores byte-compatible with the reference's
    (:func:`photon_ml_amd.io.paldb.build_paldb_index_map`, ``FeatureIndexingDriver.scala:262-291``).
  * ``photon-client/.../data/avro/NameAndTermFeatureBagsDriver.scala`` +
    ``NameAndTermFeatureSetContainer.scala`` — write, per feature bag, the set of ``name\\tterm`` lines under
    ``<output>/<bag>`` (read back by ``--feature-bags-directory`` of the GAME drivers).

Both scan the Avro files with the native columnar decoder (feature keys are interned once per distinct key).

Usage::

    python -m photon_ml_amd.cli.feature_tools index --input-data-directories in/ --root-output-directory idx/ \\
        --num-storage-partitions 4 --feature-shard-configurations name=global,feature.bags=features
    python -m photon_ml_amd.cli.feature_tools bags --input-data-directories in/ --root-output-directory bags/ \\
        --feature-bags-keys features,userFeatures
"""
from __future__ import annotations

import argparse
import os
import sys
from collections import OrderedDict
from typing import Dict, List, Sequence

from ..constants import split_feature_key
from ..io.avro import avro_files, native
from ..io.index_map import build_offheap_index_map
from ..io.paldb import build_paldb_index_map
from ..utils.timing import Timed
from .game_training import process_output_dir, resolve_paths
from .params import parse_bool, parse_feature_shard_configuration, split_list


def scan_bag_keys(paths: Sequence[str], bags: Sequence[str]) -> Dict[str, List[str]]:
    """Distinct feature keys per bag over all Avro files (sorted)."""
    files = avro_files(list(paths))
    if not files:
        raise FileNotFoundError(f"No Avro files found at {paths}")
    cols = native().read_columnar(files, ["response", "label"], "weight", "offset", "uid", "metadataMap",
                                  list(bags), [], "\u0001")
    vocab = list(cols["vocab"])
    out = {}
    for b in bags:
        if b not in cols["bags"]:
            raise ValueError(f"Feature section not found: {b}")
        import numpy as np
        used = np.unique(cols["bags"][b][1])
        out[b] = sorted(vocab[i] for i in used)
    return out


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="feature-tools", description=__doc__.split("\n")[0])
    sub = p.add_subparsers(dest="cmd", required=True)
    for name in ("index", "bags"):
        s = sub.add_parser(name)
        s.add_argument("--input-data-directories", action="append", required=True)
        s.add_argument("--input-data-date-range")
        s.add_argument("--input-data-days-range")
        s.add_argument("--root-output-directory", required=True)
        s.add_argument("--override-output-directory", type=parse_bool, default=False)
        s.add_argument("--application-name", default="Feature-Indexing-Job")
        if name == "index":
            s.add_argument("--num-storage-partitions", type=int, default=1)
            s.add_argument("--minimum-input-partitions", type=int, default=1)
            s.add_argument("--feature-shard-configurations", action="append", required=True)
            s.add_argument("--index-format", default="native", choices=["native", "paldb"],
                           help="native: this framework's mmap stores; paldb: PalDB V1 stores readable by the "
                                "reference's PalDBIndexMap (paldb-partition-<shard>-<i>.dat)")
        else:
            s.add_argument("--feature-bags-keys", required=True)
    return p


def run_indexing(a) -> Dict[str, object]:
    process_output_dir(a.root_output_directory, a.override_output_directory)
    os.makedirs(a.root_output_directory, exist_ok=True)
    shards = OrderedDict()
    for s in a.feature_shard_configurations:
        shards.update(parse_feature_shard_configuration(s))
    if a.num_storage_partitions <= 0:
        raise ValueError("num storage partitions must be > 0")
    paths = resolve_paths(a.input_data_directories, a.input_data_date_range, a.input_data_days_range)
    all_bags = sorted({b for cfg in shards.values() for b in cfg.feature_bags})
    with Timed("Scan feature keys"):
        keys = scan_bag_keys(paths, all_bags)
    maps = {}
    for sid, cfg in shards.items():
        ks = sorted({k for b in cfg.feature_bags for k in keys[b]})
        with Timed(f"Build index map {sid}"):
            build = build_paldb_index_map if getattr(a, "index_format", "native") == "paldb" else \
                build_offheap_index_map
            maps[sid] = build(ks, a.root_output_directory, sid, a.num_storage_partitions,
                              add_intercept=cfg.has_intercept)
    return maps


def run_bags(a) -> Dict[str, List[str]]:
    process_output_dir(a.root_output_directory, a.override_output_directory)
    os.makedirs(a.root_output_directory, exist_ok=True)
    paths = resolve_paths(a.input_data_directories, a.input_data_date_range, a.input_data_days_range)
    bags = split_list([a.feature_bags_keys])
    keys = scan_bag_keys(paths, bags)
    for b, ks in keys.items():
        with open(os.path.join(a.root_output_directory, b), "w") as f:
            for k in ks:
                n, t = split_feature_key(k)
                f.write(f"{n}\t{t}\n")
    return keys


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    (run_indexing if a.cmd == "index" else run_bags)(a)
    return 0


def indexing_main(argv=None) -> int:
    """``feature-indexing`` launcher: the reference's FeatureIndexingDriver
    (photon-client/.../index/FeatureIndexingDriver.scala:298-320) = ``feature_tools index``."""
    return main(["index"] + list(sys.argv[1:] if argv is None else argv))


def bags_main(argv=None) -> int:
    """``feature-bags`` launcher: the reference's NameAndTermFeatureBagsDriver
    (photon-client/.../data/avro/NameAndTermFeatureBagsDriver.scala:198-220) = ``feature_tools bags``."""
    return main(["bags"] + list(sys.argv[1:] if argv is None else argv))


if __name__ == "__main__":
    sys.exit(main())
