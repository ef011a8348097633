"""Reader for PalDB V1 feature-index stores (the reference's off-heap index map format).

Reference: ``photon-api/.../index/PalDBIndexMap.scala:43-278`` and ``PalDBIndexMapLoader.scala:25-111``. The
reference keeps, per feature shard, ``numPartitions`` PalDB stores ``paldb-partition-<namespace>-<i>.dat``; each
store holds BOTH directions — feature key (``name + "\\u0001" + term``) -> local index and local index -> feature
key — and the global index of a feature is its local index plus the number of features in the preceding
partitions (``_offsets(i) = sum of size/2``). A feature lives in partition ``nonNegativeMod(key.hashCode, n)``
(Spark ``HashPartitioner``).

PalDB itself is an external Java library; this module reads its on-disk V1 layout directly (derived from the
stores shipped with the reference, e.g. ``GameIntegTest/input/feature-indexes``):

* header: ``writeUTF("PALDB_V1")``, ``long`` timestamp, ``int`` key count, ``int`` number of key lengths,
  ``int`` max key length; per key length ``{int length, int count, int slots, int slotSize, int indexOffset,
  long dataOffset}``; ``int`` serializer count (0); ``int`` index start; ``long`` data start (all big-endian);
* index: per key length, ``slots`` slots of ``slotSize`` bytes = serialized key + LongPacker varint offset into
  the data section (0 = empty slot);
* data: varint value length + serialized value;
* serialization: small ints as one code byte (``-1 .. 8`` -> ``4 .. 13``), ``14`` + one unsigned byte,
  ``15`` / ``16`` + varint (negative / positive), strings ``103`` + varint length + one varint per UTF-16 unit.

**Production path: native** (``io/csrc/index_map.cpp``, ``pml_pdb_*``). :class:`PalDBIndexMap` mmaps the stores
and answers batched ``get_indices`` / ``get_feature_names`` with PalDB's own lookup — serialize the key, slot
``(murmur3_32(serialized key, seed 42) & 0x7fffffff) % slots`` of its key-length block, linear probing until the key
or an empty slot (offset 0) — one C call per batch, partition by Java ``String.hashCode`` in C++; nothing is
deserialised at open, no Python dict is built, and processes on one host share the page cache (the reference keeps
the stores open off-heap the same way). :func:`build_paldb_index_map` partitions, sorts, de-duplicates and writes
every store in C++ (``pml_pdb_build``).

The writer layout (reference ``PalDBIndexMapBuilder.scala:27-98``, ``FeatureIndexingDriver.scala:262-291``):
``slots = round(count / 0.75)`` per key length, each key length's data stream starts with one reserved byte (offset
0 marks an empty slot) and a slot is the serialized key plus the varint data offset, padded to the block's widest
offset. The pure-Python :func:`write_store` / :func:`read_store` below are the byte-level specification the native
code is tested against (``tests/test_paldb.py``: both writers reproduce the reference's shipped stores byte for byte;
the native reader agrees with the slot-enumerating Python reader on every key); they are not on the load path.
"""
from __future__ import annotations

import ctypes
import math
import mmap
import os
import struct
from typing import Dict, List, Optional, Tuple

import numpy as np

from .index_map import IndexMap

MAGIC = "PALDB_V1"
_STRING = 103


def _java_hash(s: str) -> int:
    h = 0
    for ch in s.encode("utf-16-be").decode("utf-16-be"):
        for unit in _utf16_units(ch):
            h = (31 * h + unit) & 0xFFFFFFFF
    return h - (1 << 32) if h >= (1 << 31) else h


def _utf16_units(ch: str):
    o = ord(ch)
    if o < 0x10000:
        return (o,)
    o -= 0x10000
    return (0xD800 + (o >> 10), 0xDC00 + (o & 0x3FF))


def partition_of(key: str, n_partitions: int) -> int:
    """Spark ``HashPartitioner.getPartition`` of a feature key (``nonNegativeMod(key.hashCode, n)``)."""
    m = _java_hash(key) % n_partitions
    return m + n_partitions if m < 0 else m


def _varint(buf, pos: int) -> Tuple[int, int]:
    """LongPacker.unpackLong: 7 bits per byte, little-endian groups, high bit = continuation."""
    result, shift = 0, 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if b & 0x80 == 0:
            return result, pos
        shift += 7
        if shift > 63:
            raise ValueError("malformed PalDB varint")


def _deserialize(buf, pos: int):
    code = buf[pos]
    pos += 1
    if 4 <= code <= 13:
        return code - 5, pos
    if code == 14:
        return buf[pos], pos + 1
    if code in (15, 16):
        v, pos = _varint(buf, pos)
        return (-v if code == 15 else v), pos
    if code == _STRING:
        n, pos = _varint(buf, pos)
        units = []
        for _ in range(n):
            u, pos = _varint(buf, pos)
            units.append(u)
        return struct.pack(f">{n}H", *units).decode("utf-16-be"), pos
    raise ValueError(f"unsupported PalDB serialization code {code}")


def murmur3_32(data: bytes, seed: int = 42) -> int:
    """MurmurHash3 x86 32-bit (PalDB ``HashUtils``: seed 42, then ``& 0x7fffffff``)."""
    c1, c2, m = 0xCC9E2D51, 0x1B873593, 0xFFFFFFFF
    h = seed & m
    nb = len(data) // 4
    for (k,) in struct.iter_unpack("<I", data[:4 * nb]):
        k = (k * c1) & m
        k = ((k << 15) | (k >> 17)) & m
        h ^= (k * c2) & m
        h = ((h << 13) | (h >> 19)) & m
        h = (h * 5 + 0xE6546B64) & m
    tail = data[4 * nb:]
    if tail:
        k = 0
        for i, b in enumerate(tail):
            k |= b << (8 * i)
        k = (k * c1) & m
        k = ((k << 15) | (k >> 17)) & m
        h ^= (k * c2) & m
    h ^= len(data)
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & m
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & m
    return h ^ (h >> 16)


def _pack_varint(v: int) -> bytes:
    """LongPacker.packLong (non-negative)."""
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _serialize(v) -> bytes:
    """PalDB StorageSerialization of an int or a string (the only types an index store holds)."""
    if isinstance(v, (int, np.integer)) and not isinstance(v, bool):
        v = int(v)
        if -1 <= v <= 8:
            return bytes([v + 5])
        if 0 <= v < 255:                                        # 255 itself is packed (reference stores)
            return bytes([14, v])
        return bytes([15]) + _pack_varint(-v) if v < 0 else bytes([16]) + _pack_varint(v)
    if isinstance(v, str):
        units = struct.unpack(f">{len(v.encode('utf-16-be')) // 2}H", v.encode("utf-16-be"))
        return bytes([_STRING]) + _pack_varint(len(units)) + b"".join(_pack_varint(u) for u in units)
    raise TypeError(f"PalDB index stores hold ints and strings, not {type(v).__name__}")


def write_store(path: str, items, timestamp_ms: Optional[int] = None) -> None:
    """Write ``items`` (iterable of (key, value) pairs; ints / strings; keys distinct) as one PalDB V1 store.
    Values are laid out per key length in insertion order."""
    import time as _time
    blocks: Dict[int, list] = {}
    for k, v in items:
        kb, vb = _serialize(k), _serialize(v)
        blocks.setdefault(len(kb), []).append((kb, vb))
    lengths = sorted(blocks)
    meta, index_parts, data_parts = [], [], []
    index_off = data_off = 0
    for L in lengths:
        ents = blocks[L]
        count = len(ents)
        slots = int(math.floor(count / 0.75 + 0.5))           # Java Math.round(count / loadFactor)
        data = bytearray(b"\x00")                             # offset 0 = empty slot
        offs = []
        for _, vb in ents:
            offs.append(len(data))
            data += _pack_varint(len(vb)) + vb
        slot_size = L + max(len(_pack_varint(o)) for o in offs)
        index = bytearray(slots * slot_size)
        used = bytearray(slots)
        for (kb, _), o in zip(ents, offs):
            s = (murmur3_32(kb) & 0x7FFFFFFF) % slots
            while used[s]:
                s = (s + 1) % slots
            used[s] = 1
            rec = kb + _pack_varint(o)
            index[s * slot_size:s * slot_size + len(rec)] = rec
        meta.append((L, count, slots, slot_size, index_off, data_off))
        index_parts.append(bytes(index))
        data_parts.append(bytes(data))
        index_off += len(index)
        data_off += len(data)
    magic = MAGIC.encode("utf-8")
    head = bytearray(struct.pack(">H", len(magic)) + magic)
    head += struct.pack(">q", int(_time.time() * 1000) if timestamp_ms is None else int(timestamp_ms))
    head += struct.pack(">iii", sum(m[1] for m in meta), len(meta), max(lengths, default=0))
    for L, count, slots, slot_size, io, do in meta:
        head += struct.pack(">iiiiiq", L, count, slots, slot_size, io, do)
    head += struct.pack(">i", 0)                                # no custom serializers
    index_start = len(head) + 12
    head += struct.pack(">iq", index_start, index_start + index_off)
    tmp = path + ".tmp"
    with open(tmp, "wb") as fh:
        fh.write(bytes(head))
        for b in index_parts:
            fh.write(b)
        for b in data_parts:
            fh.write(b)
    os.replace(tmp, path)


def _nul_join(strings) -> bytes:
    """Strings as one NUL-separated UTF-8 blob (the native ABI's batch format)."""
    # a key holding a NUL shifts the separator count: the native side checks it against the key count and fails
    return "\0".join(strings).encode("utf-8", "surrogatepass")


def _lib():
    from .index_map import _imlib
    return _imlib()


def _err() -> str:
    return _lib().pml_pdb_last_error().decode("utf-8", "replace")


def write_store_native(path: str, keys_in_index_order, timestamp_ms: Optional[int] = None) -> None:
    """One two-way store (key i -> i, i -> key i) written by the native writer (same bytes as :func:`write_store`
    of those items)."""
    import time as _time
    keys = list(keys_in_index_order)
    blob = _nul_join(keys)
    ts = int(_time.time() * 1000) if timestamp_ms is None else int(timestamp_ms)
    if _lib().pml_pdb_write_store(path.encode(), blob, len(blob), len(keys), ts) != 0:
        raise OSError(f"PalDB store {path}: {_err()}")


def build_paldb_index_map(keys, directory: str, namespace: str, n_partitions: int = 1,
                          add_intercept: bool = True, timestamp_ms: Optional[int] = None) -> "PalDBIndexMap":
    """FeatureIndexingDriver with PalDB output: distinct feature keys hash-partitioned like Spark's
    ``HashPartitioner`` (Java ``String.hashCode``), local indices 0.. in sorted key order per partition, one store per
    partition holding both directions (key -> local index, local index -> key). Partitioning, sorting,
    de-duplication and the store bytes are native (``pml_pdb_build``, partitions written in parallel)."""
    import time as _time
    from .index_map import INTERCEPT_KEY
    keys = list(keys)
    if add_intercept:
        keys.append(INTERCEPT_KEY)              # de-duplicated natively
    os.makedirs(directory, exist_ok=True)
    blob = _nul_join(keys)
    paths = _nul_join(store_file(directory, namespace, p) for p in range(n_partitions))
    sizes = np.zeros(n_partitions, dtype=np.int64)
    ts = int(_time.time() * 1000) if timestamp_ms is None else int(timestamp_ms)
    rc = _lib().pml_pdb_build(blob, len(blob), len(keys), n_partitions, paths, len(paths), ts, sizes.ctypes.data)
    if rc != 0:
        raise OSError(f"PalDB index build in {directory}: {_err()} ({rc})")
    return PalDBIndexMap(directory, namespace, n_partitions)


def partitions_native(keys, n_partitions: int) -> np.ndarray:
    """:func:`partition_of` of many keys in one native call."""
    keys = list(keys)
    blob = _nul_join(keys)
    out = np.empty(len(keys), dtype=np.int32)
    if _lib().pml_pdb_partitions(blob, len(blob), len(keys), n_partitions, out.ctypes.data) != 0:
        raise ValueError(_err())
    return out


def read_store(path: str) -> Dict[object, object]:
    """All key -> value pairs of one PalDB V1 store."""
    with open(path, "rb") as fh:
        buf = mmap.mmap(fh.fileno(), 0, access=mmap.ACCESS_READ)
    try:
        (n,) = struct.unpack_from(">H", buf, 0)
        magic = bytes(buf[2:2 + n]).decode("utf-8")
        if magic != MAGIC:
            raise ValueError(f"{path}: not a PalDB V1 store (header {magic!r})")
        pos = 2 + n + 8
        key_count, n_lengths, _max_len = struct.unpack_from(">iii", buf, pos)
        pos += 12
        blocks = []
        for _ in range(n_lengths):
            klen, count, slots, slot_size, idx_off = struct.unpack_from(">iiiii", buf, pos)
            (data_off,) = struct.unpack_from(">q", buf, pos + 20)
            blocks.append((klen, count, slots, slot_size, idx_off, data_off))
            pos += 28
        (n_ser,) = struct.unpack_from(">i", buf, pos)
        if n_ser != 0:
            raise ValueError(f"{path}: custom PalDB serializers are not supported")
        pos += 4
        (index_start,) = struct.unpack_from(">i", buf, pos)
        (data_start,) = struct.unpack_from(">q", buf, pos + 4)
        out: Dict[object, object] = {}
        for klen, count, slots, slot_size, idx_off, data_off in blocks:
            base = index_start + idx_off
            found = 0
            for s in range(slots):
                sp = base + s * slot_size
                off, _ = _varint(buf, sp + klen)
                if off == 0:
                    continue
                key, kend = _deserialize(buf, sp)
                if kend != sp + klen:
                    raise ValueError(f"{path}: key length mismatch in slot {s}")
                vp = data_start + data_off + off
                vlen, vp = _varint(buf, vp)
                val, vend = _deserialize(buf, vp)
                if vend != vp + vlen:
                    raise ValueError(f"{path}: value length mismatch in slot {s}")
                out[key] = val
                found += 1
            if found != count:
                raise ValueError(f"{path}: {found} keys of length {klen}, header says {count}")
        if len(out) != key_count:
            raise ValueError(f"{path}: {len(out)} keys, header says {key_count}")
        return out
    finally:
        buf.close()


def store_file(directory: str, namespace: str, partition: int) -> str:
    return os.path.join(directory, f"paldb-partition-{namespace}-{partition}.dat")


def has_paldb_stores(directory: str, namespace: str) -> bool:
    return os.path.exists(store_file(directory, namespace, 0))


class PalDBIndexMap(IndexMap):
    """Read-only index map over the ``n_partitions`` PalDB stores of one namespace (feature shard), mmap'd and
    queried natively (``PalDBIndexMap.scala:75-93`` getIndex, ``118-160`` getFeatureName). Global index = local
    index + the preceding partitions' sizes (store key count / 2)."""

    def __init__(self, directory: str, namespace: str, n_partitions: int):
        self.n_partitions = n_partitions
        self.directory, self.namespace = directory, namespace
        paths = _nul_join(store_file(directory, namespace, p) for p in range(n_partitions))
        self._h = _lib().pml_pdb_open(paths, len(paths), n_partitions)
        if not self._h:
            raise ValueError(f"PalDB index {directory}/{namespace}: {_err()}")
        self._dim = int(_lib().pml_pdb_size(self._h))
        self.offsets: List[int] = [int(_lib().pml_pdb_part_offset(self._h, p)) for p in range(n_partitions)]

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                _lib().pml_pdb_close(h)
            except Exception:  # pragma: no cover - interpreter shutdown
                pass
            self._h = None

    def get_index(self, key: str) -> int:
        return int(self.get_indices([key])[0])

    def get_indices(self, keys) -> np.ndarray:
        keys = list(keys)
        out = np.empty(len(keys), dtype=np.int64)
        if not keys:
            return out
        blob = _nul_join(keys)
        if _lib().pml_pdb_get_indices(self._h, blob, len(blob), len(keys), out.ctypes.data) != 0:
            raise ValueError(f"PalDB lookup: {_err()}")
        return out

    def get_feature_names(self, indices) -> List[Optional[str]]:
        """Feature keys of many global indices (None where absent), one native call."""
        idx = np.ascontiguousarray(np.asarray(indices, dtype=np.int64).reshape(-1))
        n = idx.size
        if n == 0:
            return []
        found = np.zeros(n, dtype=np.uint8)
        lib = _lib()
        ptr = ctypes.c_char_p()
        size = int(lib.pml_pdb_get_names(self._h, idx.ctypes.data, n, ctypes.byref(ptr), found.ctypes.data))
        try:
            names = ctypes.string_at(ptr, size).decode("utf-8", "surrogatepass").split("\0")
        finally:
            lib.pml_pdb_free(ptr)
        if found.all():
            return names
        return [k if f else None for k, f in zip(names, found)]

    def get_feature_name(self, idx: int) -> Optional[str]:
        return self.get_feature_names([idx])[0] if 0 <= idx < self._dim else None

    @property
    def feature_dimension(self) -> int:
        return self._dim

    def __len__(self) -> int:
        return self._dim

    def keys_in_order(self) -> List[str]:
        return self.get_feature_names(np.arange(self._dim, dtype=np.int64))
