"""Host emulation of the block schedule used by ``glm_kernels.hip`` (CPU tests of the decomposition).

Runs the exact per-block arithmetic order of the kernels in numpy: 8-aligned windows, masked products,
per-block segment sums, long-segment pieces summed in order by the combine step. Used to test
``pml_build_blocks`` (every segment covered exactly once, windows inside the padded streams) without a GPU.
"""
from __future__ import annotations

import ctypes

import numpy as np

from .native import check, require_glm_lib

VEC = 8


def build_blocks(seg_ptr: np.ndarray, nb: int = None, maxseg: int = None):
    lib = require_glm_lib()
    seg_ptr = np.ascontiguousarray(seg_ptr, dtype=np.int32)
    nseg = len(seg_ptr) - 1
    nb = nb or lib.pml_nb()
    maxseg = maxseg or lib.pml_maxseg()
    nblk, nlong, npart = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    check(lib.pml_build_blocks(seg_ptr.ctypes.data, nseg, nb, maxseg, None, ctypes.byref(nblk), None, None,
                               ctypes.byref(nlong), ctypes.byref(npart)), "count")
    blk = np.zeros(max(5 * nblk.value, 5), dtype=np.int32)
    long_seg = np.zeros(max(nlong.value, 1), dtype=np.int32)
    long_ptr = np.zeros(nlong.value + 1, dtype=np.int32)
    check(lib.pml_build_blocks(seg_ptr.ctypes.data, nseg, nb, maxseg, blk.ctypes.data, ctypes.byref(nblk),
                               long_seg.ctypes.data, long_ptr.ctypes.data, ctypes.byref(nlong),
                               ctypes.byref(npart)), "build")
    return blk[: 5 * nblk.value].reshape(-1, 5), long_seg[: nlong.value], long_ptr, npart.value


def segment_sums(seg_ptr, idx, val, x, nb=None, maxseg=None, square=False):
    """Emulate one segmented-stream pass; returns per-segment sums (fp64) and the block table."""
    blk, long_seg, long_ptr, npart = build_blocks(seg_ptr, nb, maxseg)
    nseg = len(seg_ptr) - 1
    nnz = int(seg_ptr[-1])
    pad = ((nnz + 7) // 8) * 8 + 8
    idx_p = np.zeros(pad, dtype=np.int64)
    idx_p[:nnz] = idx
    val_p = np.zeros(pad)
    val_p[:nnz] = val
    out = np.zeros(nseg)
    seen = np.zeros(nseg, dtype=np.int64)
    parts = np.zeros(max(npart, 1))
    nb_eff = nb or require_glm_lib().pml_nb()
    for seg_lo, seg_hi, nz_lo, nz_hi, part in blk:
        lo = nz_lo & ~(VEC - 1)
        hi = (nz_hi + VEC - 1) & ~(VEC - 1)
        assert hi <= pad and hi - lo <= nb_eff + 2 * VEC
        e = np.arange(lo, hi)
        inr = (e >= nz_lo) & (e < nz_hi)
        v = val_p[lo:hi] ** 2 if square else val_p[lo:hi]
        prod = np.where(inr, v * x[np.where(inr, idx_p[lo:hi], 0)], 0.0)
        if part >= 0:
            parts[part] = prod.sum()
            continue
        for s in range(seg_lo, seg_hi):
            out[s] = prod[seg_ptr[s] - lo: seg_ptr[s + 1] - lo].sum()
            seen[s] += 1
    for L, s in enumerate(long_seg):
        out[s] = parts[long_ptr[L]:long_ptr[L + 1]].sum()
        seen[s] += 1
    assert np.all(seen == 1), "segment not covered exactly once"
    return out, blk
