"""Feature index maps (feature key ``name\\u0001term`` <-> column index).

Reference: ``photon-api/.../index/{IndexMap,DefaultIndexMap,DefaultIndexMapLoader,PalDBIndexMap,
PalDBIndexMapBuilder,PalDBIndexMapLoader}.scala`` (``featureDimension = max index + 1``), the feature-bag text lists
of ``photon-client/.../data/avro/NameAndTermFeatureSetContainer.scala`` (intercept appended LAST when requested)
and ``photon-client/.../index/IdentityIndexMapLoader.scala`` (LibSVM: index = integer name, intercept last).

* :class:`DefaultIndexMap` — in-memory dict (small/medium vocabularies).
* :class:`OffHeapIndexMap` — one or more memory-mapped hash-table partitions built by the native
  ``io/csrc/index_map.cpp`` (the PalDB replacement): ``global index = local index + partition offset`` with keys
  hash-partitioned across partitions exactly like ``PalDBIndexMap`` (partition = stable hash(name) % P).
"""
from __future__ import annotations

import ctypes
import os
import zlib
from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np

from ..constants import DELIMITER, INTERCEPT_KEY, feature_key, split_feature_key
from ..ops.build import StaleLibraryError, expected_id, verified_path


class IndexMap:
    def get_index(self, key: str) -> int:
        raise NotImplementedError

    def get_feature_name(self, idx: int) -> Optional[str]:
        raise NotImplementedError

    @property
    def feature_dimension(self) -> int:
        raise NotImplementedError

    def __contains__(self, key: str) -> bool:
        return self.get_index(key) >= 0

    def __len__(self) -> int:
        raise NotImplementedError

    def get_indices(self, keys: Sequence[str]) -> np.ndarray:
        return np.array([self.get_index(k) for k in keys], dtype=np.int64)

    @property
    def intercept_index(self) -> Optional[int]:
        i = self.get_index(INTERCEPT_KEY)
        return i if i >= 0 else None

    def keys_in_order(self) -> List[str]:
        return [self.get_feature_name(i) for i in range(self.feature_dimension)]


class DefaultIndexMap(IndexMap):
    def __init__(self, key_to_index: Optional[Dict[str, int]] = None, index_to_key: Optional[List[str]] = None):
        """From a key -> index dict, or from the distinct keys in index order (``index_to_key``: the dict is then
        built on the first key lookup -- a reader that maps its vocabulary by sorting needs none)."""
        if index_to_key is not None:
            self.index_to_key = list(index_to_key)
            self._dim = len(self.index_to_key)
            self._k2i = None
            return
        self._k2i = dict(key_to_index or {})
        self._dim = (max(self._k2i.values()) + 1) if self._k2i else 0
        self.index_to_key = [None] * self._dim
        for k, i in self._k2i.items():
            self.index_to_key[i] = k

    @property
    def key_to_index(self) -> Dict[str, int]:
        if self._k2i is None:
            self._k2i = {k: i for i, k in enumerate(self.index_to_key)}
        return self._k2i

    @staticmethod
    def from_keys(keys: Iterable[str], add_intercept: bool = False) -> "DefaultIndexMap":
        ks = list(dict.fromkeys(keys))
        if add_intercept and INTERCEPT_KEY not in ks:
            ks.append(INTERCEPT_KEY)
        return DefaultIndexMap(index_to_key=ks)

    def get_index(self, key):
        return self.key_to_index.get(key, -1)

    def get_feature_name(self, idx):
        return self.index_to_key[idx] if 0 <= idx < self._dim else None

    def get_indices(self, keys):
        g = self.key_to_index.get
        return np.fromiter((g(k, -1) for k in keys), dtype=np.int64, count=len(keys))

    @property
    def feature_dimension(self):
        return self._dim

    def __len__(self):
        return len(self.key_to_index)

    def save_text(self, path: str):
        """One ``name\\tterm`` per line (feature-bag list format), in index order."""
        with open(path, "w") as f:
            for k in self.index_to_key:
                n, t = split_feature_key(k)
                f.write(f"{n}\t{t}\n")


class IdentityIndexMap(IndexMap):
    """LibSVM index map: name = integer index; optional intercept at the last index."""

    def __init__(self, dim: int, use_intercept: bool):
        self._dim = dim
        self.use_intercept = use_intercept

    def get_index(self, key):
        if self.use_intercept and key == INTERCEPT_KEY:
            return self._dim - 1
        name, _ = split_feature_key(key)
        try:
            i = int(name)
        except ValueError:
            return -1
        return i if 0 <= i < self._dim else -1

    def get_feature_name(self, idx):
        if self.use_intercept and idx == self._dim - 1:
            return INTERCEPT_KEY
        return feature_key(str(idx), "") if 0 <= idx < self._dim else None

    @property
    def feature_dimension(self):
        return self._dim

    def __len__(self):
        return self._dim


# ----------------------------------------------------------------------------------------------------------------
_IMLIB = None


def _imlib():
    global _IMLIB
    if _IMLIB is None:
        path = verified_path("cpp", "indexmap")   # stale builds are rebuilt or refused (ops/build.py build ids)
        lib = ctypes.CDLL(str(path))
        lib.pml_build_id.restype = ctypes.c_char_p
        if lib.pml_build_id().decode() != expected_id("cpp", "indexmap"):
            raise StaleLibraryError(f"{path}: loaded build id {lib.pml_build_id().decode()} != the tree's sources")
        lib.pml_im_build.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_char_p]
        lib.pml_im_open.argtypes = [ctypes.c_char_p]
        lib.pml_im_open.restype = ctypes.c_void_p
        lib.pml_im_close.argtypes = [ctypes.c_void_p]
        lib.pml_im_size.argtypes = [ctypes.c_void_p]
        lib.pml_im_size.restype = ctypes.c_int64
        lib.pml_im_lookup.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int64]
        lib.pml_im_lookup.restype = ctypes.c_int64
        lib.pml_im_lookup_many.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int64,
                                           ctypes.c_void_p]
        lib.pml_im_name.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_char_p, ctypes.c_int64]
        lib.pml_im_name.restype = ctypes.c_int64
        # PalDB V1 stores (io/paldb.py)
        vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32
        lib.pml_pdb_last_error.restype = ctypes.c_char_p
        lib.pml_pdb_partitions.argtypes = [ctypes.c_char_p, i64, i64, i32, vp]
        lib.pml_pdb_write_store.argtypes = [ctypes.c_char_p, ctypes.c_char_p, i64, i64, i64]
        lib.pml_pdb_build.argtypes = [ctypes.c_char_p, i64, i64, i32, ctypes.c_char_p, i64, i64, vp]
        lib.pml_pdb_open.argtypes = [ctypes.c_char_p, i64, i32]
        lib.pml_pdb_open.restype = vp
        lib.pml_pdb_close.argtypes = [vp]
        lib.pml_pdb_size.argtypes = [vp]
        lib.pml_pdb_size.restype = i64
        lib.pml_pdb_part_offset.argtypes = [vp, i32]
        lib.pml_pdb_part_offset.restype = i64
        lib.pml_pdb_get_indices.argtypes = [vp, ctypes.c_char_p, i64, i64, vp]
        lib.pml_pdb_get_names.argtypes = [vp, vp, i64, ctypes.POINTER(ctypes.c_char_p), vp]
        lib.pml_pdb_get_names.restype = i64
        lib.pml_pdb_free.argtypes = [ctypes.c_char_p]
        _IMLIB = lib
    return _IMLIB


def _pack(keys: Sequence[str]):
    bs = [k.encode("utf-8") for k in keys]
    offs = np.zeros(len(bs) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(b) for b in bs])
    return b"".join(bs), offs


def partition_of(name: str, n_partitions: int) -> int:
    """Stable hash partition of a feature NAME (PalDB stores are partitioned by name)."""
    return zlib.crc32(name.encode("utf-8")) % n_partitions


def store_path(directory: str, namespace: str, partition: int) -> str:
    return os.path.join(directory, f"pml-index-partition-{namespace}-{partition}.idx")


def build_offheap_index_map(keys: Sequence[str], directory: str, namespace: str, n_partitions: int = 1,
                            add_intercept: bool = True) -> "OffHeapIndexMap":
    """Partition keys by feature name, build one mmap store per partition (FeatureIndexingDriver)."""
    keys = list(dict.fromkeys(keys))
    if add_intercept and INTERCEPT_KEY not in keys:
        keys.append(INTERCEPT_KEY)
    os.makedirs(directory, exist_ok=True)
    parts: List[List[str]] = [[] for _ in range(n_partitions)]
    for k in keys:
        parts[partition_of(split_feature_key(k)[0], n_partitions)].append(k)
    lib = _imlib()
    for p, ks in enumerate(parts):
        ks.sort()
        blob, offs = _pack(ks)
        rc = lib.pml_im_build(blob, offs.ctypes.data, len(ks), store_path(directory, namespace, p).encode())
        if rc != 0:
            raise RuntimeError(f"index map build failed ({rc})")
    return OffHeapIndexMap(directory, namespace, n_partitions)


class OffHeapIndexMap(IndexMap):
    def __init__(self, directory: str, namespace: str, n_partitions: int):
        lib = _imlib()
        self.n_partitions = n_partitions
        self.handles = []
        for p in range(n_partitions):
            h = lib.pml_im_open(store_path(directory, namespace, p).encode())
            if not h:
                raise FileNotFoundError(store_path(directory, namespace, p))
            self.handles.append(h)
        sizes = [lib.pml_im_size(h) for h in self.handles]
        self.offsets = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        self._dim = int(self.offsets[-1])

    def __del__(self):
        try:
            lib = _imlib()
            for h in self.handles:
                lib.pml_im_close(h)
        except Exception:  # pragma: no cover
            pass

    def get_index(self, key):
        p = partition_of(split_feature_key(key)[0], self.n_partitions)
        b = key.encode("utf-8")
        i = _imlib().pml_im_lookup(self.handles[p], b, len(b))
        return int(self.offsets[p] + i) if i >= 0 else -1

    def get_indices(self, keys):
        out = np.full(len(keys), -1, dtype=np.int64)
        parts = np.array([partition_of(split_feature_key(k)[0], self.n_partitions) for k in keys], dtype=np.int64)
        lib = _imlib()
        for p in range(self.n_partitions):
            sel = np.nonzero(parts == p)[0]
            if len(sel) == 0:
                continue
            blob, offs = _pack([keys[i] for i in sel])
            res = np.empty(len(sel), dtype=np.int64)
            lib.pml_im_lookup_many(self.handles[p], blob, offs.ctypes.data, len(sel), res.ctypes.data)
            out[sel] = np.where(res >= 0, res + self.offsets[p], -1)
        return out

    def get_feature_name(self, idx):
        if idx < 0 or idx >= self._dim:
            return None
        p = int(np.searchsorted(self.offsets, idx, side="right") - 1)
        local = idx - int(self.offsets[p])
        lib = _imlib()
        n = lib.pml_im_name(self.handles[p], local, None, 0)
        buf = ctypes.create_string_buffer(max(n, 1))
        lib.pml_im_name(self.handles[p], local, buf, n)
        return buf.raw[:n].decode("utf-8")

    @property
    def feature_dimension(self):
        return self._dim

    def __len__(self):
        return self._dim


# ----------------------------------------------------------------------------------------------------------------
def read_feature_bag_file(path: str) -> List[str]:
    """Feature-bag list file(s): one ``name\\tterm`` (or ``name``) per line -> feature keys."""
    files = [os.path.join(path, f) for f in sorted(os.listdir(path)) if not f.startswith((".", "_"))] \
        if os.path.isdir(path) else [path]
    keys = []
    for fp in files:
        with open(fp) as f:
            for line in f:
                line = line.rstrip("\n")
                if not line:
                    continue
                parts = line.split("\t")
                if len(parts) > 2:
                    raise ValueError(f"Unexpected entry {line!r} in {fp}")
                keys.append(feature_key(parts[0], parts[1] if len(parts) == 2 else ""))
    return keys


def index_map_from_feature_bags(bags_dir: str, bags: Sequence[str], add_intercept: bool) -> DefaultIndexMap:
    """NameAndTermFeatureSetContainer.getFeatureNameAndTermToIndexMap (sorted union for determinism)."""
    keys = set()
    for b in bags:
        keys.update(read_feature_bag_file(os.path.join(bags_dir, b)))
    return DefaultIndexMap.from_keys(sorted(keys), add_intercept)


def open_index_map(directory: str, namespace: str, n_partitions: int = 1) -> IndexMap:
    """Off-heap index map of one namespace (feature shard): the reference's PalDB stores
    (``paldb-partition-<ns>-<i>.dat``, mmap'd and probed natively, :mod:`photon_ml_amd.io.paldb`) when present, else
    the native mmap stores written by the feature-indexing driver."""
    from .paldb import PalDBIndexMap, has_paldb_stores
    if has_paldb_stores(directory, namespace):
        return PalDBIndexMap(directory, namespace, n_partitions)
    return OffHeapIndexMap(directory, namespace, n_partitions)
