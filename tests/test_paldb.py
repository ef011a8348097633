"""PalDB V1 index-store reader (io/paldb.py) on the reference's own stores.

Reference expectations: ``photon-api/src/test/scala/com/linkedin/photon/ml/index/PalDBIndexMapTest.scala``
(exact name -> index values of the heart stores, 2 partitions, with and without intercept); the GAME
integration-test stores ``GameIntegTest/input/feature-indexes/paldb-partition-shard{1,2,3}-0.dat`` and the
duplicate-feature Avro input of ``AvroDataReaderIntegTest.scala:85``. The heart stores and the duplicate-feature
Avro file are copied into ``tests/fixtures``; the (larger) GAME stores are read from the reference tree.
"""
import os

import numpy as np
import pytest

from photon_ml_amd.constants import INTERCEPT_KEY
from photon_ml_amd.io.index_map import open_index_map
from photon_ml_amd.io.paldb import PalDBIndexMap, partition_of, read_store

FIX = os.path.join(os.path.dirname(__file__), "fixtures")
GAME = "/root/reference/photon-client/src/integTest/resources/GameIntegTest/input"
DELIM = "\u0001"


def key(name, term=""):
    return name + DELIM + term


# PalDBIndexMapTest.testNoInterceptMap / testWithInterceptMap
NO_ICPT = {"1": 0, "2": 7, "3": 5, "4": 11, "5": 6, "6": 9, "7": 3, "8": 8, "9": 1, "10": 4, "11": 12, "12": 2,
           "13": 10}
WITH_ICPT = {"1": 0, "2": 8, "3": 5, "4": 12, "5": 6, "6": 10, "7": 2, "8": 9, "9": 1, "10": 4, "11": 13, "12": 3,
             "13": 11}


def test_heart_store_without_intercept():
    m = PalDBIndexMap(os.path.join(FIX, "paldb_heart"), "global", 2)
    assert len(m) == 13 and m.feature_dimension == 13
    assert m.get_index(INTERCEPT_KEY) == -1
    for name, idx in NO_ICPT.items():
        assert m.get_index(key(name)) == idx
        assert m.get_feature_name(idx) == key(name)
    assert m.get_feature_name(13) is None


def test_heart_store_with_intercept_and_opener():
    m = open_index_map(os.path.join(FIX, "paldb_heart_icpt"), "global", 2)
    assert isinstance(m, PalDBIndexMap) and len(m) == 14
    assert m.get_index(INTERCEPT_KEY) == 7
    for name, idx in WITH_ICPT.items():
        assert m.get_index(key(name)) == idx and m.get_feature_name(idx) == key(name)
    np.testing.assert_array_equal(m.get_indices([key("2"), "nope", INTERCEPT_KEY]), [8, -1, 7])


def test_partitioning_is_spark_hash_partitioner():
    """Every feature key sits in partition nonNegativeMod(key.hashCode, n) (Spark HashPartitioner)."""
    for d in ("paldb_heart", "paldb_heart_icpt"):
        for p in range(2):
            kv = read_store(os.path.join(FIX, d, f"paldb-partition-global-{p}.dat"))
            names = [k for k in kv if isinstance(k, str)]
            assert names and all(partition_of(k, 2) == p for k in names)


@pytest.mark.skipif(not os.path.isdir(GAME), reason="reference GAME integration-test inputs not present")
def test_game_integration_stores():
    maps = {s: PalDBIndexMap(os.path.join(GAME, "feature-indexes"), s, 1) for s in ("shard1", "shard2", "shard3")}
    for m in maps.values():
        n = len(m)
        names = m.keys_in_order()
        assert len(set(names)) == n and all(m.get_index(k) == i for i, k in enumerate(names))
        assert m.get_index(INTERCEPT_KEY) >= 0
    k1, k2, k3 = (set(maps[s].keys_in_order()) for s in ("shard1", "shard2", "shard3"))
    song = {key("s", str(i)) for i in range(30)}
    user = {key("u", str(i)) for i in range(30)}
    # shard3: song features + intercept; shard2: global + user features; shard1: global + user + song features
    assert k3 == song | {INTERCEPT_KEY}
    assert k2 == k1 - song and user <= k2 and not (song & k2)
    # every name of the feature-bag lists that the indexing run saw in the data is indexed
    lists = os.path.join(GAME, "feature-lists")

    def bag(name):
        return {line.rstrip("\n").replace("\t", DELIM) for line in open(os.path.join(lists, name), encoding="utf-8")
                if line.strip()}
    assert bag("songFeatures") <= k3 and bag("userFeatures") <= k2
    assert len(bag("features") & k1) > 0.99 * len(k1 - song - user - {INTERCEPT_KEY})


def test_duplicate_feature_records_are_rejected():
    """AvroDataReaderIntegTest.testReadDuplicateFeatures: a record listing one feature twice fails the read."""
    from photon_ml_amd.io.data_reader import AvroDataReader, DuplicateFeatureError, FeatureShardConfiguration
    path = os.path.join(FIX, "duplicate-features-yahoo-music-train.avro")
    with pytest.raises(DuplicateFeatureError):
        AvroDataReader().read(path, {"global": FeatureShardConfiguration(["features"], True)})
    # the other bags of the same file are clean
    data, _ = AvroDataReader().read(path, {"user": FeatureShardConfiguration(["userFeatures"], True)})
    assert data.n_rows == 6


def test_legacy_driver_trains_with_reference_paldb_index(tmp_path):
    """DriverIntegTest with an off-heap index map: the heart PalDB stores (with intercept) drive the feature
    indexing of the heart Avro input; the learned model is laid out in the store's index order."""
    from photon_ml_amd.cli import driver as drv
    ref = "/root/reference/photon-client/src/integTest/resources/DriverIntegTest/input/heart.avro"
    train = ref if os.path.exists(ref) else os.path.join(FIX, "heart.avro")
    args = ["--training-data-directory", train, "--output-directory", str(tmp_path / "o"), "--task",
            "LOGISTIC_REGRESSION", "--num-iterations", "30", "--device", "cpu", "--offheap-indexmap-dir",
            os.path.join(FIX, "paldb_heart_icpt"), "--offheap-indexmap-num-partitions", "2"]
    d = drv.Driver(drv.build_parser().parse_args(args)).run()
    assert d.train_data.n_features == 14
    models = drv.read_text_model(str(tmp_path / "o" / drv.LEARNED_MODELS_TEXT))
    (lam, coefs), = models.items()
    assert len(coefs) == 14


# ---------------------------------------------------------------------------------------------------------------
# PalDB writer (io/paldb.py write_store / build_paldb_index_map; reference PalDBIndexMapBuilder.scala:27-98)
def _rebuild(path, out):
    import struct
    from photon_ml_amd.io.paldb import write_store
    kv = read_store(path)
    by_index = sorted((v, k) for k, v in kv.items() if isinstance(k, str))
    with open(path, "rb") as fh:
        buf = fh.read()
    ts = struct.unpack_from(">q", buf, 10)[0]        # after writeUTF("PALDB_V1")
    write_store(out, [(k, i) for i, k in by_index] + [(i, k) for i, k in by_index], ts)
    with open(out, "rb") as fh:
        return buf, fh.read()


@pytest.mark.parametrize("path", [os.path.join(FIX, "paldb_heart", "paldb-partition-global-0.dat"),
                                  os.path.join(FIX, "paldb_heart", "paldb-partition-global-1.dat"),
                                  os.path.join(FIX, "paldb_heart_icpt", "paldb-partition-global-0.dat"),
                                  os.path.join(GAME, "feature-indexes", "paldb-partition-shard1-0.dat"),
                                  os.path.join(GAME, "feature-indexes", "paldb-partition-shard3-0.dat")])
def test_writer_reproduces_reference_stores_bytewise(path, tmp_path):
    """Rewriting a reference store's contents (keys inserted by index, its timestamp) gives the SAME bytes: slot
    hash (murmur3, seed 42), slot counts, slot widths, int / string serialisation, data layout."""
    if not os.path.exists(path):
        pytest.skip("reference store not present")
    ref, out = _rebuild(path, str(tmp_path / "s.dat"))
    assert out == ref


def test_built_index_map_is_readable_and_probe_consistent(tmp_path):
    """build_paldb_index_map: Spark-hash partitions, both directions per store, and every key reachable by PalDB's
    own lookup (hash slot, linear probing until an empty slot) — what the reference's reader does."""
    import struct
    from photon_ml_amd.io.paldb import _serialize, _varint, build_paldb_index_map, murmur3_32, store_file
    keys = [key(f"f{i % 97}", str(i)) for i in range(3000)] + [key("été", "x"), key("n", "")]
    m = build_paldb_index_map(keys, str(tmp_path), "global", 3, add_intercept=True)
    assert len(m) == len(set(keys)) + 1 and m.get_index(INTERCEPT_KEY) >= 0
    assert sorted(m.get_index(k) for k in keys + [INTERCEPT_KEY]) == list(range(len(m)))
    assert all(m.get_feature_name(m.get_index(k)) == k for k in keys)
    assert open_index_map(str(tmp_path), "global", 3).get_index(keys[5]) == m.get_index(keys[5])
    for p in range(3):
        path = store_file(str(tmp_path), "global", p)
        buf = open(path, "rb").read()
        n_lengths = struct.unpack_from(">i", buf, 22)[0]
        blocks = [struct.unpack_from(">iiiiiq", buf, 30 + 28 * i) for i in range(n_lengths)]
        index_start = struct.unpack_from(">i", buf, 30 + 28 * n_lengths + 4)[0]
        info = {b[0]: b for b in blocks}
        for k, v in read_store(path).items():
            kb = _serialize(k)
            L, count, slots, slot_size, io, _ = info[len(kb)]
            s = (murmur3_32(kb) & 0x7FFFFFFF) % slots
            for _probe in range(slots):
                sp = index_start + io + s * slot_size
                off, _ = _varint(buf, sp + L)
                assert off != 0, f"key {k!r} not reachable by probing"
                if buf[sp:sp + L] == kb:
                    break
                s = (s + 1) % slots
            assert partition_of(k if isinstance(k, str) else v, 3) == p


def test_indexing_driver_writes_paldb(tmp_path):
    """The feature-indexing driver with --index-format paldb writes paldb-partition-<shard>-<i>.dat stores that the
    loaders (open_index_map) pick up."""
    from photon_ml_amd.cli.feature_tools import main as ft_main
    out = tmp_path / "idx"
    ft_main(["index", "--input-data-directories", os.path.join(FIX, "heart.avro"), "--root-output-directory",
             str(out), "--num-storage-partitions", "2", "--index-format", "paldb",
             "--feature-shard-configurations", "name=global,feature.bags=features"])
    assert os.path.exists(out / "paldb-partition-global-0.dat")
    m = open_index_map(str(out), "global", 2)
    assert isinstance(m, PalDBIndexMap) and len(m) == 14       # 13 heart features + intercept


# ---------------------------------------------------------------------------------------------------------------
# Native PalDB path (io/csrc/index_map.cpp pml_pdb_*): the production reader / writer, checked against the
# slot-enumerating Python reader (read_store) and the Python writer (write_store), the byte-level specification.
STORES = [os.path.join(FIX, "paldb_heart", "paldb-partition-global-0.dat"),
          os.path.join(FIX, "paldb_heart", "paldb-partition-global-1.dat"),
          os.path.join(FIX, "paldb_heart_icpt", "paldb-partition-global-0.dat"),
          os.path.join(FIX, "paldb_heart_icpt", "paldb-partition-global-1.dat"),
          os.path.join(GAME, "feature-indexes", "paldb-partition-shard1-0.dat"),
          os.path.join(GAME, "feature-indexes", "paldb-partition-shard2-0.dat"),
          os.path.join(GAME, "feature-indexes", "paldb-partition-shard3-0.dat")]


@pytest.mark.parametrize("path", STORES)
def test_native_writer_reproduces_reference_stores_bytewise(path, tmp_path):
    import struct
    from photon_ml_amd.io.paldb import write_store_native
    if not os.path.exists(path):
        pytest.skip("reference store not present")
    kv = read_store(path)
    by_index = [k for _, k in sorted((v, k) for k, v in kv.items() if isinstance(k, str))]
    ref = open(path, "rb").read()
    ts = struct.unpack_from(">q", ref, 10)[0]
    out = str(tmp_path / "n.dat")
    write_store_native(out, by_index, ts)
    assert open(out, "rb").read() == ref


@pytest.mark.parametrize("path", STORES)
def test_native_reader_agrees_with_slot_enumeration(path):
    """Every key of a reference store found by PalDB's probe in the native reader, with the value the Python
    slot-enumerating reader decodes; absent keys give -1 / None."""
    if not os.path.exists(path):
        pytest.skip("reference store not present")
    d, f = os.path.split(path)
    ns = f[len("paldb-partition-"):-len("-0.dat")]
    n_parts = len([x for x in os.listdir(d) if x.startswith(f"paldb-partition-{ns}-")])
    m = PalDBIndexMap(d, ns, n_parts)
    p = int(f[:-4].rsplit("-", 1)[1])
    kv = read_store(path)
    names = [k for k in kv if isinstance(k, str)]
    got = m.get_indices(names)
    np.testing.assert_array_equal(got, [m.offsets[p] + kv[k] for k in names])
    assert m.get_feature_names(got) == names
    assert m.get_indices(["not-a-feature" + DELIM, ""]).tolist() == [-1, -1]
    assert m.get_feature_names([-1, len(m), len(m) + 5]) == [None, None, None]


def test_native_build_matches_python_writer_and_partitions(tmp_path):
    """pml_pdb_build (partition, sort, de-duplicate, write) gives the bytes of the Python writer over the same
    sorted partitions; partitions follow Java String.hashCode (incl. non-BMP characters and empty terms)."""
    from photon_ml_amd.io.paldb import (build_paldb_index_map, partitions_native, store_file, write_store)
    keys = [key(f"f{i % 53}", str(i)) for i in range(5000)] + [key("été", "x"), key("n", ""), key("😀", "t"),
                                                               key("f1", "1")]   # one duplicate
    m = build_paldb_index_map(keys, str(tmp_path / "n"), "g", 4, add_intercept=True, timestamp_ms=123456789)
    distinct = sorted(set(keys) | {INTERCEPT_KEY})
    assert len(m) == len(distinct)
    parts = partitions_native(distinct, 4)
    assert parts.tolist() == [partition_of(k, 4) for k in distinct]
    for p in range(4):
        ks = sorted(k for k, q in zip(distinct, parts) if q == p)
        ref = str(tmp_path / f"py{p}.dat")
        write_store(ref, [(k, i) for i, k in enumerate(ks)] + [(i, k) for i, k in enumerate(ks)], 123456789)
        assert open(store_file(str(tmp_path / "n"), "g", p), "rb").read() == open(ref, "rb").read()
    idx = m.get_indices(distinct)
    assert sorted(idx.tolist()) == list(range(len(m)))
    assert m.get_feature_names(idx) == distinct
    assert m.keys_in_order() == [distinct[i] for i in np.argsort(idx)]


def test_native_paldb_scale(tmp_path):
    """200k keys over 2 partitions: build, open and batched lookups well under a second each (the 10M-key record is
    profiles/paldb_native_r6.md)."""
    import time
    keys = [key(f"feat{i % 1000}", f"t{i}") for i in range(200_000)]
    t = time.time()
    from photon_ml_amd.io.paldb import build_paldb_index_map
    build_paldb_index_map(keys, str(tmp_path), "s", 2)
    t_build = time.time() - t
    t = time.time()
    m = PalDBIndexMap(str(tmp_path), "s", 2)
    t_open = time.time() - t
    t = time.time()
    idx = m.get_indices(keys)
    t_get = time.time() - t
    assert len(m) == 200_001 and (idx >= 0).all() and len(set(idx.tolist())) == 200_000
    assert t_open < 0.1 and t_get < 2.0 and t_build < 5.0, (t_build, t_open, t_get)
