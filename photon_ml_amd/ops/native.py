"""ctypes bindings of the native HIP libraries (C ABI).

The libraries are loaded AFTER ``import torch`` so that their ``libamdhip64.so.7`` dependency resolves to the
HIP runtime torch already loaded (one runtime, one device context, torch-owned memory and streams).
On a GPU box the HIP path is mandatory: :func:`require_glm_lib` raises if the library is missing instead of
silently falling back to the torch reference.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path
from typing import Optional

import numpy as np
import torch  # noqa: F401  (must precede loading the HIP libraries)

from .build import StaleLibraryError, expected_id, lib_path, verified_path

c_int = ctypes.c_int
c_double = ctypes.c_double
c_void_p = ctypes.c_void_p
P_int = ctypes.POINTER(ctypes.c_int)


class SegChunkDesc(ctypes.Structure):
    _fields_ = [
        ("blk", c_void_p), ("nblk", c_int),
        ("seg_ptr", c_void_p), ("nseg", c_int),
        ("idx", c_void_p), ("val", c_void_p),
        ("long_seg", c_void_p), ("long_ptr", c_void_p), ("nlong", c_int), ("npart", c_int),
    ]


class TLNarrow(ctypes.Structure):
    """Narrow-section streams of one chunk (16-bit packs, values, one int32 base per round), plus the wide
    section's per-round key bases (``wbase``, NULL when the wide packs hold absolute keys)."""
    _fields_ = [("pack", c_void_p), ("val", c_void_p), ("base", c_void_p), ("wbase", c_void_p)]


class TLFwdDesc(ctypes.Structure):
    _fields_ = [("blk", c_void_p), ("nblk", c_int), ("rbits", c_int), ("pack", c_void_p), ("val", c_void_p),
                ("il", c_int), ("nar", TLNarrow), ("live", c_void_p)]


class TLFwdMultiDesc(ctypes.Structure):
    """``ptrs``: 5 stream pointers per chunk {pack, val, narrow pack, narrow val, narrow base}."""
    _fields_ = [("blk", c_void_p), ("nblk", c_int), ("rbits", c_int), ("ptrs", c_void_p), ("il", c_int),
                ("live", c_void_p)]


class TLTMultiDesc(ctypes.Structure):
    _fields_ = [("items", c_void_p), ("nitems", c_int), ("cbits", c_int), ("ptrs", c_void_p),
                ("mt_tiles", c_void_p), ("mt_ptr", c_void_p), ("nmt", c_int), ("dim", c_int), ("cu", c_void_p),
                ("ncu", c_int), ("nparts_total", c_int), ("il", c_int), ("live", c_void_p), ("live_mt", c_void_p)]


class CmpArgs(ctypes.Structure):
    """Arguments of the row-sampled tiled-chunk copy (``tl_compact_kernel``, ops/csrc/game_kernels.hip)."""
    _fields_ = [("units", c_void_p), ("col_e", c_int), ("row_col", c_int), ("seg", c_void_p), ("nseg", c_int),
                ("sbits", c_int), ("key_is_row", c_int), ("pack", c_void_p), ("val", c_void_p),
                ("npack", c_void_p), ("nval", c_void_p), ("nbase", c_void_p), ("keep", c_void_p),
                ("seg_cnt", c_void_p), ("seg_first", c_void_p), ("unit_lo", c_void_p), ("opack", c_void_p),
                ("oval", c_void_p)]


class TLTDesc(ctypes.Structure):
    _fields_ = [
        ("items", c_void_p), ("nitems", c_int), ("cbits", c_int), ("pack", c_void_p), ("val", c_void_p),
        ("mt_tiles", c_void_p), ("mt_ptr", c_void_p), ("nmt", c_int), ("dim", c_int),
        ("cu", c_void_p), ("ncu", c_int), ("nparts_total", c_int), ("il", c_int), ("nar", TLNarrow),
        ("live", c_void_p), ("live_mt", c_void_p),
    ]


_LIBS = {}


def _load(name: str, auto_build: bool = True) -> Optional[ctypes.CDLL]:
    """Load ``libpml_<name>.so``. The in-tree library must carry the build id of the tree's sources
    (``ops/build.py``): a stale one is rebuilt when hipcc is available and otherwise raises
    :class:`~photon_ml_amd.ops.build.StaleLibraryError` — it is never loaded. None when the library is missing
    and cannot be built (CPU-only installs). ``PML_GLM_LIB`` / ``PML_RE_LIB`` name explicit A/B or profiling
    builds, which are loaded as given."""
    if name in _LIBS:
        return _LIBS[name]
    override = {"glm": "PML_GLM_LIB", "re": "PML_RE_LIB"}.get(name)
    if override and os.environ.get(override):
        path = Path(os.environ[override])
        want = None
    else:
        try:
            path = verified_path("hip", name, auto_build=auto_build)
        except FileNotFoundError:
            _LIBS[name] = None
            return None
        want = expected_id("hip", name)
    lib = ctypes.CDLL(str(path), mode=ctypes.RTLD_GLOBAL)
    if want is not None:
        lib.pml_build_id.restype = ctypes.c_char_p
        got = lib.pml_build_id().decode()
        if got != want:
            raise StaleLibraryError(f"{path}: loaded build id {got} != {want} of the tree's sources")
    _LIBS[name] = lib
    return lib


def glm_lib() -> Optional[ctypes.CDLL]:
    lib = _load("glm")
    if lib is not None and not getattr(lib, "_pml_typed", False):
        lib.pml_build_blocks.argtypes = [c_void_p, c_int, c_int, c_int, c_void_p, P_int, c_void_p, c_void_p,
                                         P_int, P_int]
        lib.pml_seg_fwd.argtypes = [c_int, ctypes.POINTER(SegChunkDesc), c_void_p, c_int, c_int, c_double,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                    c_void_p, c_void_p, c_void_p]
        lib.pml_seg_t.argtypes = [c_int, ctypes.POINTER(SegChunkDesc), c_void_p, c_int, c_void_p, c_void_p,
                                  c_void_p]
        lib.pml_reduce_stats.argtypes = [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p]
        lib.pml_lds_add_order_probe.argtypes = [c_void_p, c_void_p, c_int, c_void_p]
        lib.pml_lds_add_order_probe.restype = c_int
        lib.pml_tl_fwd.argtypes = [c_int, ctypes.POINTER(TLFwdDesc), c_void_p, c_int, c_int, c_double, c_void_p,
                                   c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p]
        lib.pml_tl_t.argtypes = [c_int, ctypes.POINTER(TLTDesc), c_void_p, c_int, c_void_p, c_void_p, c_void_p]
        lib.pml_tl_config.argtypes = [c_int, c_int, c_int, c_int]
        lib.pml_tl_t_multi.argtypes = [c_int, ctypes.POINTER(TLTMultiDesc), c_void_p, c_int, c_void_p, c_void_p,
                                       c_void_p]
        lib.pml_tl_fwd_multi.argtypes = [c_int, ctypes.POINTER(TLFwdMultiDesc), c_void_p, c_int, c_int, c_double,
                                         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                         c_void_p]
        lib.pml_segdot.argtypes = [c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p]
        lib.pml_segdot_long.argtypes = [c_void_p, c_void_p, c_int, c_void_p, c_int, ctypes.c_longlong, c_void_p,
                                        c_void_p, c_void_p]
        lib.pml_seg_expand.argtypes = [c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p]
        lib.pml_seg_cg_step.argtypes = [c_void_p, c_int] + [c_void_p] * 7 + [c_double, c_void_p]
        lib.pml_bgemv.argtypes = [c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p]
        lib.pml_btrsv.argtypes = [c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p]
        lib.pml_bhv.argtypes = [c_int, c_int, c_void_p, c_void_p, c_void_p, c_double, c_void_p, c_void_p]
        lib.pml_set_ls_args.argtypes = [c_void_p, c_double, c_double]
        lib.pml_set_ls_in.argtypes = [c_void_p, c_void_p]
        lib.pml_set_gate.argtypes = [c_void_p]
        lib.pml_ls_gate.argtypes = [c_void_p, c_void_p, c_double, c_double, c_double, c_double, c_void_p, c_void_p,
                                    c_void_p]
        lib.pml_ls_gate.restype = c_int
        lib.pml_gram_grid.argtypes = [ctypes.c_longlong]
        lib.pml_gram.argtypes = [c_void_p, c_int, ctypes.c_longlong, c_void_p, c_void_p]
        lib.pml_lincomb.argtypes = [c_void_p, c_void_p, c_int, ctypes.c_longlong, c_void_p, c_void_p]
        lib.pml_lbfgs_pair.argtypes = [c_void_p] * 4 + [ctypes.c_longlong] + [c_void_p] * 6
        lib.pml_ls_dots.argtypes = [c_void_p] * 3 + [ctypes.c_longlong] + [c_void_p] * 4
        lib.pml_perm_cast.argtypes = [c_void_p, c_void_p, ctypes.c_longlong, c_int, c_void_p, c_void_p]
        lib.pml_perm_cast.restype = c_int
        lib.pml_ls_step_grad.argtypes = [c_void_p, c_void_p, c_double, c_void_p, c_void_p, c_double,
                                         ctypes.c_longlong, c_void_p, c_void_p, c_void_p]
        lib.pml_ls_step_grad.restype = c_int
        lib.pml_masked_gather.argtypes = [c_void_p, c_void_p, ctypes.c_longlong, c_void_p, c_void_p]
        lib.pml_masked_gather.restype = c_int
        lib.pml_offset_update.argtypes = [c_void_p, c_void_p, ctypes.c_longlong, c_int, c_void_p, c_void_p, c_void_p]
        lib.pml_cached_margins.argtypes = [c_void_p, c_void_p, c_double, c_int, c_void_p, ctypes.c_longlong,
                                           c_void_p, c_void_p]
        lib.pml_cached_margins.restype = c_int
        lib.pml_offset_update.restype = c_int
        lib.pml_two_loop_chain.argtypes = [c_int] + [c_void_p] * 5 + [ctypes.c_longlong] + [c_void_p] * 4 + \
            [c_int, c_void_p]
        lib.pml_two_loop_gram.argtypes = [c_int, c_void_p, c_void_p, c_void_p, ctypes.c_longlong, c_void_p, c_void_p,
                                          c_void_p, c_int, c_void_p]
        lib.pml_two_loop_gram_grid.argtypes = [ctypes.c_longlong]
        lib.pml_tl_set_deep.argtypes = [c_int, c_int]
        lib.pml_rs_set_variant.argtypes = [c_int]
        lib.pml_rs_set_variant(int(os.environ.get("PML_RS_VARIANT", "5")))
        lib.pml_ls_eval.argtypes = [c_int, c_int, c_double, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]
        lib.pml_ls_eval_multi.argtypes = [c_int, c_int, c_int, ctypes.POINTER(c_double), c_int, c_void_p, c_void_p,
                                          c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]
        lib.pml_ls_eval_multi.restype = c_int
        lib.pml_rs_tron.argtypes = [c_int, c_int] + [c_void_p] * 8 + [c_int, c_double, c_double, c_int, c_int, c_int,
                                                                      c_void_p, c_void_p, c_void_p]
        for f in ("pml_seg_fwd", "pml_seg_t", "pml_reduce_stats", "pml_build_blocks", "pml_tl_fwd", "pml_tl_t",
                  "pml_tl_maxbits", "pml_segdot", "pml_segdot_long", "pml_tl_fwd_multi", "pml_tl_t_multi", "pml_seg_cg_step",
                  "pml_seg_expand", "pml_bgemv", "pml_btrsv", "pml_bhv", "pml_rs_tron", "pml_ls_eval", "pml_gram_grid", "pml_gram",
                  "pml_lincomb", "pml_lbfgs_pair", "pml_ls_dots", "pml_two_loop_chain", "pml_two_loop_gram",
                  "pml_two_loop_gram_grid"):
            getattr(lib, f).restype = c_int
        lib.pml_set_config.argtypes = [c_int, c_int, c_int, c_int]
        lib._pml_typed = True
        configure()
    return lib


# Kernel configuration defaults (tuned on MI355X, see profiles/): forward = vector layout + 8192-entry LDS hot
# table of the most frequent features; transpose = strided layout. Env overrides for experiments:
# PML_FWD_STRIDED, PML_T_STRIDED, PML_HOT_N, PML_FWD_GRID.
KERNEL_CONFIG = {"fwd_strided": 0, "t_strided": 0, "hot_n": 0, "fwd_grid": 1024, "tl_acc64": 1, "tl_waves": 2,
                 "tl_waves_t": 4, "tl_pipe": 0, "tl_pipe_t": 0, "tl_multi": 1, "tl_deep": 0, "tl_deep_t": 0}


def configure(**kw):
    KERNEL_CONFIG.update({k: v for k, v in kw.items() if v is not None})
    for k in list(KERNEL_CONFIG):
        env = os.environ.get("PML_" + k.upper())
        if env is not None and k not in kw:
            KERNEL_CONFIG[k] = int(env)
    lib = _LIBS.get("glm")
    if lib is not None:
        lib.pml_set_config(KERNEL_CONFIG["fwd_strided"], KERNEL_CONFIG["t_strided"], KERNEL_CONFIG["hot_n"],
                           KERNEL_CONFIG["fwd_grid"])
        lib.pml_tl_config(KERNEL_CONFIG["tl_acc64"], KERNEL_CONFIG["tl_waves"], KERNEL_CONFIG["tl_waves_t"],
                          (KERNEL_CONFIG["tl_pipe"] & 3) | ((KERNEL_CONFIG["tl_pipe_t"] & 3) << 2))
        lib.pml_tl_set_deep(KERNEL_CONFIG["tl_deep"], KERNEL_CONFIG["tl_deep_t"])
    return dict(KERNEL_CONFIG)


def tl_experiment_build() -> bool:
    """True when the loaded GLM library is the experiment build (-DPML_TL_EXPERIMENT): only there do the stream
    pipeline / wave-count / accumulation knobs select A/B kernel variants."""
    lib = glm_lib()
    return lib is not None and bool(lib.pml_tl_experiment())


def require_glm_lib() -> ctypes.CDLL:
    lib = glm_lib()
    if lib is None:
        raise RuntimeError(
            f"native GLM kernel library missing ({lib_path('hip', 'glm')}); run python -m photon_ml_amd.ops.build")
    return lib


def segdot(a: torch.Tensor, b: Optional[torch.Tensor], ptr: torch.Tensor, mode: int = 0) -> torch.Tensor:
    """Per-segment sum of a*b (mode 0) / a (1) / |a| (2) over contiguous segments ``ptr`` (int64, device).
    fp64, deterministic; CUDA tensors use the HIP kernel, CPU tensors a cumsum-free reduceat."""
    nseg = ptr.numel() - 1
    if a.device.type != "cuda":
        import numpy as np
        v = (a * b if mode == 0 else (a if mode == 1 else a.abs())).detach().cpu().numpy()
        p = ptr.cpu().numpy()
        out = np.zeros(nseg)
        nz = p[1:] > p[:-1]
        if v.size and nz.any():
            out[nz] = np.add.reduceat(v, p[:-1][nz])
        return torch.from_numpy(out).to(a.device)
    lib = require_glm_lib()
    a = a.contiguous()
    b = a if b is None else b.contiguous()
    out = torch.empty(nseg, dtype=torch.float64, device=a.device)
    # the longest segment, measured once per segment table (one host read; the tables are built once per
    # dataset): segments longer than SEGDOT_CHUNK are split over chunk waves (pml_segdot_long)
    # cached with the tensor's version counter: an in-place change of the table (e.g. cumsum(out=ptr)) re-measures
    cached = getattr(ptr, "_pml_maxlen", None)
    if cached is not None and cached[0] == ptr._version:
        maxlen = cached[1]
    else:
        maxlen = int((ptr[1:] - ptr[:-1]).max()) if nseg else 0
        ptr._pml_maxlen = (ptr._version, maxlen)
    if maxlen > SEGDOT_CHUNK:
        n = a.numel()
        scratch = torch.empty(2 * ((n + SEGDOT_CHUNK - 1) // SEGDOT_CHUNK), dtype=torch.float64, device=a.device)
        check(lib.pml_segdot_long(a.data_ptr(), b.data_ptr(), mode, ptr.data_ptr(), nseg, n, scratch.data_ptr(),
                                  out.data_ptr(), stream_handle(a.device)), "segdot_long")
        return out
    check(lib.pml_segdot(a.data_ptr(), b.data_ptr(), mode, ptr.data_ptr(), nseg, out.data_ptr(),
                         stream_handle(a.device)), "segdot")
    return out


SEGDOT_CHUNK = 4096        # = SEGDOT_C in glm_kernels.hip


GRAM_MAXK = 22


def _fast_vecs(vs) -> bool:
    return (0 < len(vs) <= GRAM_MAXK and all(v.device.type == "cuda" and v.dtype == torch.float64
                                             and v.dim() == 1 and v.is_contiguous() for v in vs)
            and len({v.numel() for v in vs}) == 1 and len({v.device for v in vs}) == 1)


def gram(vs) -> torch.Tensor:
    """Device fp64 [k, k] matrix of all inner products of k <= 22 equal-length device vectors, ONE pass over
    them (``gram_kernel``, fp64 MFMA; 16-B aligned vectors), or None when the inputs do not qualify."""
    if not _fast_vecs(vs) or any(v.data_ptr() % 16 for v in vs):
        return None
    lib = require_glm_lib()
    k, n = len(vs), vs[0].numel()
    ptrs = (ctypes.c_void_p * k)(*[v.data_ptr() for v in vs])
    npairs = k * (k + 1) // 2
    partial = torch.empty(lib.pml_gram_grid(n), npairs, dtype=torch.float64, device=vs[0].device)
    check(lib.pml_gram(ptrs, k, n, partial.data_ptr(), stream_handle(vs[0].device)), "gram")
    tri = partial.sum(0)
    iu = torch.triu_indices(k, k, device=tri.device)
    G = torch.zeros(k, k, dtype=torch.float64, device=tri.device)
    G[iu[0], iu[1]] = tri
    return G + G.triu(1).T


def lincomb(coefs, vs):
    """sum_j coefs[j] vs[j] in one pass (``lincomb_kernel``; host coefficients), or None when not applicable."""
    if not _fast_vecs(vs):
        return None
    lib = require_glm_lib()
    k, n = len(vs), vs[0].numel()
    ptrs = (ctypes.c_void_p * k)(*[v.data_ptr() for v in vs])
    cs = (ctypes.c_double * k)(*[float(c) for c in coefs])
    out = torch.empty(n, dtype=torch.float64, device=vs[0].device)
    check(lib.pml_lincomb(ptrs, cs, k, n, out.data_ptr(), stream_handle(vs[0].device)), "lincomb")
    return out


_PAIR_SCRATCH = {}


def lbfgs_pair(x, x0, g, g0, out=None):
    """New L-BFGS history pair in one launch (``lbfgs_pair_kernel``): returns ``(s, y, out)`` with s = x - x0,
    y = g - g0 and the device vector out = [s.y, y.y, 1/s.y, s.y/y.y, g.g] (written into ``out`` when given: 5
    contiguous fp64 device values); None when the inputs do not qualify."""
    vs = (x, x0, g, g0)
    if not (x.device.type == "cuda" and all(v.device == x.device and v.dtype == torch.float64 and v.dim() == 1
                                            and v.is_contiguous() and v.numel() == x.numel() for v in vs)
            and x.numel() > 0):
        return None
    lib = require_glm_lib()
    sc = _PAIR_SCRATCH.get(x.device)
    if sc is None:
        sc = _PAIR_SCRATCH[x.device] = (torch.empty(3 * 1024, dtype=torch.float64, device=x.device),
                                        torch.zeros(1, dtype=torch.int32, device=x.device))
    s, y = torch.empty_like(x), torch.empty_like(x)
    if out is None:
        out = torch.empty(5, dtype=torch.float64, device=x.device)
    assert out.device == x.device and out.dtype == torch.float64 and out.numel() == 5 and out.is_contiguous()
    check(lib.pml_lbfgs_pair(x.data_ptr(), x0.data_ptr(), g.data_ptr(), g0.data_ptr(), x.numel(), s.data_ptr(),
                             y.data_ptr(), sc[0].data_ptr(), sc[1].data_ptr(), out.data_ptr(),
                             stream_handle(x.device)), "lbfgs_pair")
    return s, y, out


_LOSS_SCRATCH = {}


def loss_sum(loss_id: int, z: torch.Tensor, y: torch.Tensor, w: torch.Tensor,
             offsets: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """0-d device fp64 ``sum_i w_i l(z_i + o_i, y_i)`` in one fused pass (``ls_eval_kernel`` + a fixed-order block
    reduction; ``offsets`` o enter as the kernel's direction at t = 1, so z + 1.0 o rounds exactly like z + o): the
    GAME training-loss evaluation after every coordinate update, instead of ~10 torch elementwise passes. None when
    the inputs do not qualify (host tensors, other dtypes)."""
    vs = (z, y, w) if offsets is None else (z, y, w, offsets)
    if not (z.device.type == "cuda" and loss_id in (0, 1, 2, 3) and 0 < z.numel() < 2 ** 31
            and all(v.device == z.device and v.dtype == torch.float64 and v.dim() == 1 and v.is_contiguous()
                    and v.numel() == z.numel() for v in vs)):
        return None
    lib = require_glm_lib()
    sc = _LOSS_SCRATCH.get(z.device)
    if sc is None:
        sc = _LOSS_SCRATCH[z.device] = torch.empty(2 * 4096, dtype=torch.float64, device=z.device)
    out = torch.empty(2, dtype=torch.float64, device=z.device)
    zd, t = (z, 0.0) if offsets is None else (offsets, 1.0)
    check(lib.pml_ls_eval(2, z.numel(), t, int(loss_id), z.data_ptr(), zd.data_ptr(), y.data_ptr(), w.data_ptr(),
                          0, None, None, sc.data_ptr(), out.data_ptr(), stream_handle(z.device)), "loss_sum")
    return out[0]


_DOTS_SCRATCH = {}


def ls_dots(x0, g, d, out=None):
    """Device vector [g.d, d.d, x0.x0, x0.d] in one launch (``ls_dots_kernel``, deterministic last-workgroup
    reduction; into ``out`` when given); None when the inputs do not qualify."""
    vs = (x0, g, d)
    if not (d.device.type == "cuda" and all(v.device == d.device and v.dtype == torch.float64 and v.dim() == 1
                                            and v.is_contiguous() and v.numel() == d.numel() for v in vs)
            and d.numel() > 0):
        return None
    lib = require_glm_lib()
    sc = _DOTS_SCRATCH.get(d.device)
    if sc is None:
        sc = _DOTS_SCRATCH[d.device] = (torch.empty(4 * 1024, dtype=torch.float64, device=d.device),
                                        torch.zeros(1, dtype=torch.int32, device=d.device))
    if out is None:
        out = torch.empty(4, dtype=torch.float64, device=d.device)
    assert out.device == d.device and out.dtype == torch.float64 and out.numel() == 4 and out.is_contiguous()
    check(lib.pml_ls_dots(x0.data_ptr(), g.data_ptr(), d.data_ptr(), d.numel(), sc[0].data_ptr(), sc[1].data_ptr(),
                          out.data_ptr(), stream_handle(d.device)), "ls_dots")
    return out


def perm_cast(w: torch.Tensor, perm: Optional[torch.Tensor], dtype: torch.dtype) -> torch.Tensor:
    """``w[perm].to(dtype)`` (``perm`` None: ``w.to(dtype)``) in one launch (``perm_cast_kernel``): a forward
    pass's coefficient input. ``w`` fp64 device vector, ``perm`` int64, ``dtype`` float32 / float64."""
    assert w.is_cuda and w.dtype == torch.float64 and w.dim() == 1 and w.is_contiguous()
    assert dtype in (torch.float32, torch.float64)
    n = w.numel() if perm is None else perm.numel()
    if perm is not None:
        assert perm.device == w.device and perm.dtype == torch.int64 and perm.is_contiguous()
        if os.environ.get("PML_CHECK_KERNEL_INPUTS", "0") == "1" and n:
            assert 0 <= int(perm.min()) and int(perm.max()) < w.numel(), "perm_cast index out of range"
    out = torch.empty(n, dtype=dtype, device=w.device)
    check(require_glm_lib().pml_perm_cast(w.data_ptr(), None if perm is None else perm.data_ptr(), n,
                                          2 if dtype == torch.float64 else 1, out.data_ptr(), stream_handle(w.device)),
          "perm_cast")
    return out


def offset_update(base: torch.Tensor, part: torch.Tensor, o: torch.Tensor, z: Optional[torch.Tensor]) -> None:
    """In place, one pass (``offset_update_kernel``): ``o = (base + part).to(o.dtype)`` and, with ``z``,
    ``z += o_new - o_old`` in fp64. ``base``, ``part``, ``z`` fp64 and ``o`` fp32 / fp64 device vectors of one
    length."""
    n = base.numel()
    for t in (base, part, o) + (() if z is None else (z,)):
        assert t.is_cuda and t.is_contiguous() and t.numel() == n and t.device == base.device
    assert base.dtype == part.dtype == torch.float64 and o.dtype in (torch.float32, torch.float64)
    assert z is None or z.dtype == torch.float64
    check(require_glm_lib().pml_offset_update(base.data_ptr(), part.data_ptr(), n,
                                              2 if o.dtype == torch.float64 else 1, o.data_ptr(),
                                              None if z is None else z.data_ptr(), stream_handle(base.device)),
          "offset_update")


def cached_margins(z0: torch.Tensor, zd: Optional[torch.Tensor], t: float, o: Optional[torch.Tensor],
                   n: int) -> torch.Tensor:
    """``(z0[:n] + t zd[:n]) - o[:n]`` (``zd`` / ``o`` None: term left out) as a new fp64 vector in one pass
    (``cached_margins_kernel``: z0 + t zd as one fma, then the offset subtraction)."""
    for v in (z0, zd, o):
        assert v is None or (v.is_cuda and v.is_contiguous() and v.numel() >= n and v.device == z0.device)
    assert z0.dtype == torch.float64 and (zd is None or zd.dtype == torch.float64)
    assert o is None or o.dtype in (torch.float32, torch.float64)
    out = torch.empty(max(n, 1), dtype=torch.float64, device=z0.device)[:n]
    check(require_glm_lib().pml_cached_margins(z0.data_ptr(), None if zd is None else zd.data_ptr(), float(t),
                                               2 if o is None or o.dtype == torch.float64 else 1,
                                               None if o is None else o.data_ptr(), n, out.data_ptr(),
                                               stream_handle(z0.device)), "cached_margins")
    return out


def masked_gather(src: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """``out[i] = src[idx[i]]``, 0 where ``idx[i] < 0`` (``masked_gather_kernel``, one pass). ``src`` fp64 device
    vector, ``idx`` int64 (values < len(src))."""
    assert src.is_cuda and src.dtype == torch.float64 and src.is_contiguous()
    assert idx.device == src.device and idx.dtype == torch.int64 and idx.is_contiguous()
    if os.environ.get("PML_CHECK_KERNEL_INPUTS", "0") == "1" and idx.numel():
        assert int(idx.max()) < src.numel(), "masked_gather index out of range"
    out = torch.empty(idx.shape, dtype=torch.float64, device=src.device)
    check(require_glm_lib().pml_masked_gather(src.data_ptr(), idx.data_ptr(), idx.numel(), out.data_ptr(),
                                              stream_handle(src.device)), "masked_gather")
    return out


def ls_step_grad(x0: torch.Tensor, d: torch.Tensor, t: float, G: torch.Tensor, perm: Optional[torch.Tensor],
                 l2: float):
    """The accepted line-search step and its full gradient in one launch (``ls_step_grad_kernel``):
    ``x = x0 + t * d`` and ``g = G[perm] + l2 * x`` (``perm`` None: ``G``), bitwise the torch expressions. All fp64
    device vectors of one length (``G`` in the data's device column order)."""
    n = x0.numel()
    for v in (x0, d, G):
        assert v.is_cuda and v.dtype == torch.float64 and v.dim() == 1 and v.is_contiguous() and v.device == x0.device
    assert d.numel() == n and G.numel() >= n
    if perm is not None:
        assert perm.device == x0.device and perm.dtype == torch.int64 and perm.numel() == n and perm.is_contiguous()
    x, g = torch.empty_like(x0), torch.empty_like(x0)
    check(require_glm_lib().pml_ls_step_grad(x0.data_ptr(), d.data_ptr(), float(t), G.data_ptr(),
                                             None if perm is None else perm.data_ptr(), float(l2), n, x.data_ptr(),
                                             g.data_ptr(), stream_handle(x0.device)), "ls_step_grad")
    return x, g


_CHAIN_SCRATCH = {}


def two_loop(s, y, rho, gamma, g, negate: bool = False):
    """L-BFGS two-loop ``H g`` (``-H g`` with ``negate``): 2k + 1 fused step kernels (``lbfgs_step_kernel``)
    launched from C++ in one call; history vectors ``s``, ``y`` and the 0-d device scalars ``rho`` (1/s.y),
    ``gamma`` (s.y/y.y of the newest pair) stay on the device. None when the inputs do not qualify."""
    k = len(s)
    if not (k > 0 and g.device.type == "cuda" and g.dtype == torch.float64 and g.dim() == 1 and g.is_contiguous()
            and g.numel() > 0):
        return None
    if not all(v.device == g.device and v.dtype == torch.float64 and v.is_contiguous() and v.numel() == g.numel()
               for v in list(s) + list(y)):
        return None
    if not all(r.device == g.device and r.dtype == torch.float64 and r.numel() == 1 for r in list(rho) + [gamma]):
        return None
    lib = require_glm_lib()
    sc = _CHAIN_SCRATCH.get(g.device)
    if sc is None or sc[0].numel() < 2 * k:
        sc = _CHAIN_SCRATCH[g.device] = (torch.empty(max(64, 2 * k), dtype=torch.float64, device=g.device),
                                         torch.empty(1024, dtype=torch.float64, device=g.device),
                                         torch.zeros(1, dtype=torch.int32, device=g.device))
    P = ctypes.c_void_p * k
    q = torch.empty_like(g)
    check(lib.pml_two_loop_chain(k, P(*[v.data_ptr() for v in s]), P(*[v.data_ptr() for v in y]),
                                 P(*[r.data_ptr() for r in rho]), gamma.data_ptr(), g.data_ptr(), g.numel(),
                                 q.data_ptr(), sc[0].data_ptr(), sc[1].data_ptr(), sc[2].data_ptr(), int(negate),
                                 stream_handle(g.device)), "two_loop_chain")
    return q


_GRAM_LOOP_SCRATCH = {}


def two_loop_gram(s, y, g, negate: bool = False):
    """L-BFGS two-loop ``H g`` (``-H g``) by the vector-free recursion on the device: one Gram pass over the
    2k + 1 vectors [s..., y..., g], the recursion in one workgroup, one linear-combination pass (3 launches, no
    host synchronisation). History lists oldest first (as ``_History``); k <= 10. None when not applicable."""
    k = len(s)
    if not (0 < k and 2 * k + 1 <= GRAM_MAXK and len(y) == k and g.device.type == "cuda"
            and g.dtype == torch.float64 and g.dim() == 1 and g.is_contiguous() and g.numel() > 0):
        return None
    if not all(v.device == g.device and v.dtype == torch.float64 and v.is_contiguous() and v.numel() == g.numel()
               and v.data_ptr() % 16 == 0 for v in list(s) + list(y) + [g]):
        return None                    # (the MFMA Gram kernel reads 16-B pairs)
    lib = require_glm_lib()
    n = g.numel()
    kk = 2 * k + 1
    need = lib.pml_two_loop_gram_grid(n) * (kk * (kk + 1) // 2)
    sc = _GRAM_LOOP_SCRATCH.get(g.device)
    if sc is None or sc[0].numel() < need:
        sc = _GRAM_LOOP_SCRATCH[g.device] = (torch.empty(max(need, 1 << 16), dtype=torch.float64, device=g.device),
                                             torch.empty(GRAM_MAXK, dtype=torch.float64, device=g.device))
    P = ctypes.c_void_p * k
    q = torch.empty_like(g)
    check(lib.pml_two_loop_gram(k, P(*[v.data_ptr() for v in s]), P(*[v.data_ptr() for v in y]), g.data_ptr(), n,
                                q.data_ptr(), sc[0].data_ptr(), sc[1].data_ptr(), int(negate),
                                stream_handle(g.device)), "two_loop_gram")
    return q


def batched_gemv(A: torch.Tensor, x: torch.Tensor, trans: bool = False) -> torch.Tensor:
    """``y[b] = A[b] x[b]`` (or ``A[b]^T x[b]``) for a batch of small square fp64 matrices (n <= 192):
    ``bgemv_kernel`` (n <= 64, blocks staged in LDS) / ``bgemv_wide_kernel`` on the device, ``bmm`` on the host
    (and beyond 192: the library GEMM, whose first call in a process pays ~50 ms of kernel loading)."""
    if A.device.type != "cuda" or A.shape[-1] > 192 or A.shape[-1] != A.shape[-2]:
        M = A.transpose(1, 2) if trans else A
        return torch.bmm(M, x.unsqueeze(-1)).squeeze(-1)
    lib = require_glm_lib()
    A, x = A.contiguous(), x.contiguous()
    B, n, _ = A.shape
    assert A.dtype == torch.float64 and x.dtype == torch.float64 and x.shape == (B, n)
    y = torch.empty_like(x)
    check(lib.pml_bgemv(B, n, A.data_ptr(), x.data_ptr(), y.data_ptr(), int(trans), stream_handle(A.device)),
          "bgemv")
    return y


def batched_trsv(L: torch.Tensor, x: torch.Tensor, trans: bool = False,
                 out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``y[b] = L[b]^-1 x[b]`` (or ``L[b]^-T x[b]``) for a batch of lower-triangular fp64 matrices (n <= 192):
    ``btrsv_kernel`` (one wave per problem, packed triangle in LDS) on the device, ``solve_triangular`` on the
    host. ``out``: a contiguous [B, n] fp64 tensor to write ``y`` into (not aliasing ``x``)."""
    if L.device.type != "cuda" or L.shape[-1] > 192 or L.shape[-1] != L.shape[-2]:
        M = L.transpose(1, 2) if trans else L
        y = torch.linalg.solve_triangular(M, x.unsqueeze(-1), upper=trans).squeeze(-1)
        return y if out is None else out.copy_(y)
    lib = require_glm_lib()
    L, x = L.contiguous(), x.contiguous()
    B, n, _ = L.shape
    assert L.dtype == torch.float64 and x.dtype == torch.float64 and x.shape == (B, n)
    if out is not None:
        assert out.shape == x.shape and out.dtype == torch.float64 and out.is_contiguous() and out.device == x.device
        assert out.data_ptr() != x.data_ptr()
    y = torch.empty_like(x) if out is None else out
    check(lib.pml_btrsv(B, n, L.data_ptr(), x.data_ptr(), y.data_ptr(), int(trans), stream_handle(L.device)),
          "btrsv")
    return y


def batched_hv(A: torch.Tensor, dw: torch.Tensor, v: torch.Tensor, l2: float = 0.0) -> torch.Tensor:
    """``A^T (dw * (A v)) + l2 v`` per problem (fp64, n <= 64): one read of each block (``bhv_kernel``)."""
    if A.device.type != "cuda" or A.shape[-1] > 64 or A.shape[-1] != A.shape[-2]:
        xv = torch.bmm(A, v.unsqueeze(-1)).squeeze(-1)
        h = torch.bmm(A.transpose(1, 2), (dw * xv).unsqueeze(-1)).squeeze(-1)
        return h + l2 * v if l2 > 0 else h
    lib = require_glm_lib()
    A, dw, v = A.contiguous(), dw.contiguous(), v.contiguous()
    B, n, _ = A.shape
    assert A.dtype == dw.dtype == v.dtype == torch.float64 and v.shape == (B, n) and dw.shape == (B, n)
    out = torch.empty_like(v)
    check(lib.pml_bhv(B, n, A.data_ptr(), dw.data_ptr(), v.data_ptr(), float(l2), out.data_ptr(),
                      stream_handle(A.device)), "bhv")
    return out


def rs_tron(L: torch.Tensor, y: torch.Tensor, o: torch.Tensor, w: torch.Tensor, beta0: torch.Tensor, loss_id: int,
            l2: float, tol: float, max_iter: int, max_fail: int = 5, max_cg: int = 20,
            out: Optional[torch.Tensor] = None, order: Optional[torch.Tensor] = None,
            zout: Optional[torch.Tensor] = None):
    """Fused per-problem TRON over a batch of small dense GLMs (``rs_tron_kernel``): returns
    (beta, f, iters, reason). ``zout`` (contiguous fp64 [B, n]) receives the margins ``L beta`` of the solution
    (written by the kernel while L is resident). Device only; n <= 192 (n > 64: ``rs_tron_big_kernel``, one wave
    per problem); losses logistic / Poisson / squared. ``out`` (contiguous
    fp64 [B, n]) receives the solution in place (it starts from ``beta0``; ``out`` may be ``beta0``). ``order``
    (int32 permutation of the B problems): waves take consecutive problems of it -- grouping problems of similar
    iteration counts cuts the time a wave waits for its slowest problem; the results do not depend on it."""
    B, n, _ = L.shape
    lib = require_re_lib() if n > 64 else require_glm_lib()
    ts = [t.contiguous() for t in (L, y, o, w)]
    for t in ts:
        assert t.dtype == torch.float64 and t.is_cuda
    assert y.shape == (B, n) and o.shape == (B, n) and w.shape == (B, n) and beta0.shape == (B, n)
    if out is None:
        beta = beta0.to(torch.float64).contiguous().clone()
    else:
        assert out.shape == (B, n) and out.dtype == torch.float64 and out.is_contiguous()
        if out.data_ptr() != beta0.data_ptr():
            out.copy_(beta0)
        beta = out
    f = torch.empty(B, dtype=torch.float64, device=L.device)
    iters = torch.empty(B, dtype=torch.int32, device=L.device)
    reason = torch.empty(B, dtype=torch.int32, device=L.device)
    if order is not None:
        assert order.dtype == torch.int32 and order.is_cuda and order.shape == (B,) and order.is_contiguous()
        if os.environ.get("PML_CHECK_KERNEL_INPUTS", "0") == "1":   # the kernel indexes L / y / beta through it
            assert B == 0 or (int(order.min()) >= 0 and int(order.max()) < B), "rs_tron order out of range"
    if zout is not None:
        assert zout.shape == (B, n) and zout.dtype == torch.float64 and zout.is_contiguous() and zout.is_cuda
    if n > 64:
        # one wave per problem, packed L in LDS (re_kernels.hip rs_tron_big_kernel); problem order not used
        check(lib.pml_rs_tron_big(B, n, ts[0].data_ptr(), ts[1].data_ptr(), ts[2].data_ptr(), ts[3].data_ptr(),
                                  beta.data_ptr(), f.data_ptr(), iters.data_ptr(), reason.data_ptr(),
                                  None if zout is None else zout.data_ptr(), int(loss_id), float(l2), float(tol),
                                  int(max_iter), int(max_fail), int(max_cg), stream_handle(L.device)), "rs_tron_big")
        return beta, f, iters.to(torch.long), reason.to(torch.long)
    check(lib.pml_rs_tron(B, n, ts[0].data_ptr(), ts[1].data_ptr(), ts[2].data_ptr(), ts[3].data_ptr(),
                          beta.data_ptr(), f.data_ptr(), iters.data_ptr(), reason.data_ptr(), int(loss_id), float(l2),
                          float(tol), int(max_iter), int(max_fail), int(max_cg),
                          None if order is None else order.data_ptr(),
                          None if zout is None else zout.data_ptr(), stream_handle(L.device)), "rs_tron")
    return beta, f, iters.to(torch.long), reason.to(torch.long)


def seg_expand(s: torch.Tensor, ptr: torch.Tensor, n: int) -> torch.Tensor:
    """``out[i] = s[e]`` over contiguous segments ``ptr`` (length ``n`` = ptr[-1]); 8-byte or 1-byte dtypes."""
    if s.device.type != "cuda" or s.element_size() not in (1, 8):
        return torch.repeat_interleave(s, ptr[1:] - ptr[:-1], output_size=n)
    lib = require_glm_lib()
    s = s.contiguous()
    out = torch.empty(n, dtype=s.dtype, device=s.device)
    check(lib.pml_seg_expand(ptr.data_ptr(), ptr.numel() - 1, s.data_ptr(), out.data_ptr(), s.element_size(),
                             stream_handle(s.device)), "seg_expand")
    return out


def seg_cg_step(ptr: torch.Tensor, step: torch.Tensor, r: torch.Tensor, d: torch.Tensor, Hd: torch.Tensor,
                rtr: torch.Tensor, on: torch.Tensor, delta: torch.Tensor, l2: float = 0.0) -> None:
    """One truncated-CG iteration for every entity segment, in place (``seg_cg_step_kernel``): updates
    ``step``, ``r``, ``d`` (fp64, concatenated segments), ``rtr`` (fp64 per entity) and ``on`` (uint8 per entity,
    cleared when the step hits the trust-region boundary ``delta``). ``Hd`` is the data term of the
    Hessian-vector product; ``l2 * d`` is added on the fly. CPU tensors: same arithmetic in torch."""
    nseg = ptr.numel() - 1
    if step.device.type == "cuda":
        lib = require_glm_lib()
        for t in (step, r, d, Hd, rtr, on, delta):
            assert t.is_contiguous()
        assert on.dtype == torch.uint8 and rtr.dtype == torch.float64 and step.dtype == torch.float64
        check(lib.pml_seg_cg_step(ptr.data_ptr(), nseg, step.data_ptr(), r.data_ptr(), d.data_ptr(), Hd.data_ptr(),
                                  rtr.data_ptr(), on.data_ptr(), delta.data_ptr(), float(l2),
                                  stream_handle(step.device)),
              "seg_cg_step")
        return
    ent = torch.repeat_interleave(torch.arange(nseg), ptr[1:] - ptr[:-1])
    sd = lambda a, b: segdot(a, b, ptr, 0)
    Hd = Hd + l2 * d if l2 else Hd
    act = on.bool()
    dhd, std_, sts, dtd = sd(d, Hd), sd(step, d), sd(step, step), sd(d, d)
    alpha = rtr / torch.where(dhd == 0, torch.ones_like(dhd), dhd)
    trial = step + alpha[ent] * d
    hit = torch.sqrt(sd(trial, trial).clamp(min=0)) > delta
    dsq = delta * delta
    rad = torch.sqrt((std_ * std_ + dtd * (dsq - sts)).clamp(min=0))
    tau = torch.where(std_ >= 0, (dsq - sts) / (std_ + rad).clamp(min=1e-300), (rad - std_) / dtd.clamp(min=1e-300))
    a = torch.where(act, torch.where(hit, tau, alpha), torch.zeros_like(alpha))
    step.add_(a[ent] * d)
    r.sub_(a[ent] * Hd)
    rn = sd(r, r)
    move = act & ~hit
    beta = rn / torch.where(rtr == 0, torch.ones_like(rtr), rtr)
    d.copy_(torch.where(move[ent], r + beta[ent] * d, d))
    rtr.copy_(torch.where(move, rn, rtr))
    on.copy_((act & ~hit).to(torch.uint8))


def game_lib() -> Optional[ctypes.CDLL]:
    """Scoring (K5/K6) and MFMA dense kernels (``ops/csrc/game_kernels.hip``)."""
    lib = _load("game")
    if lib is not None and not getattr(lib, "_pml_typed", False):
        lib.pml_score_rows.argtypes = [c_void_p, c_void_p, c_void_p, ctypes.c_longlong, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_void_p]
        lib.pml_gemm_nt.argtypes = [c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p, c_int,
                                    c_void_p]
        lib.pml_spmm_rows.argtypes = [c_void_p, c_void_p, c_void_p, ctypes.c_longlong, c_void_p, c_int, c_void_p,
                                      c_void_p]
        lib.pml_downsample.argtypes = [c_int, c_void_p, c_void_p, c_void_p, ctypes.c_longlong, ctypes.c_ulonglong,
                                       c_double, c_int, c_void_p, c_void_p]
        lib.pml_seg_gram.argtypes = [c_int, c_int, c_int, ctypes.c_longlong] + [c_void_p] * 8
        lib.pml_batched_chol.argtypes = [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]
        lib.pml_batched_chol.restype = c_int
        lib.pml_seg_gram_set_s.argtypes = [c_int]
        lib.pml_rs_primal.argtypes = [c_int, c_int] + [c_void_p] * 9 + [c_int]
        lib.pml_rs_primal.restype = c_int
        lib.pml_csr_gather_rows.argtypes = [c_int, c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_longlong,
                                            c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]
        lib.pml_csr_gather_rows.restype = c_int
        lib.pml_key_hist.argtypes = [c_int, c_void_p, ctypes.c_longlong, ctypes.c_longlong, c_void_p, c_void_p]
        lib.pml_key_hist.restype = c_int
        lib.pml_tl_compact.argtypes = [c_int, c_int, ctypes.POINTER(CmpArgs), c_void_p]
        lib.pml_tl_compact.restype = c_int
        for f in ("pml_score_rows", "pml_gemm_nt", "pml_spmm_rows", "pml_downsample"):
            getattr(lib, f).restype = c_int
        lib._pml_typed = True
    return lib


def require_game_lib() -> ctypes.CDLL:
    lib = game_lib()
    if lib is None:
        raise RuntimeError(
            f"native GAME kernel library missing ({lib_path('hip', 'game')}); run python -m photon_ml_amd.ops.build")
    return lib


def score_rows(indptr: torch.Tensor, col32: torch.Tensor, val: torch.Tensor, w: torch.Tensor,
               ent: Optional[torch.Tensor] = None, eptr: Optional[torch.Tensor] = None,
               efeat: Optional[torch.Tensor] = None) -> torch.Tensor:
    """K5 / K6 scoring of a device CSR shard (``score_rows_kernel``): ``x_i . w`` (fixed effect) or, with the
    entity-major model CSR (``ent`` row -> entity index or -1, ``eptr``, sorted ``efeat``, values ``w``),
    ``x_i . w_{e(i)}``. fp64, deterministic."""
    lib = require_game_lib()
    n = indptr.numel() - 1
    assert indptr.dtype == torch.int64 and col32.dtype == torch.int32 and val.dtype == torch.float64
    assert w.dtype == torch.float64 and indptr.is_cuda and col32.is_cuda and val.is_cuda and w.is_cuda
    if ent is not None:
        assert ent.dtype == torch.int32 and ent.numel() == n and eptr.dtype == torch.int64
        assert efeat.dtype == torch.int32 and efeat.numel() == w.numel()
    out = torch.empty(n, dtype=torch.float64, device=val.device)
    p = lambda t: None if t is None else t.data_ptr()
    check(lib.pml_score_rows(indptr.data_ptr(), col32.data_ptr(), val.data_ptr(), n, w.data_ptr(), p(ent), p(eptr),
                             p(efeat), out.data_ptr(), stream_handle(val.device)), "score_rows")
    return out


def key_histogram(keys: torch.Tensor, nbins: int) -> torch.Tensor:
    """``torch.bincount(keys, minlength=nbins)`` (int64) for keys in [0, nbins) with very hot keys
    (``key_hist_kernel``: per-workgroup LDS aggregation, one global atomic per distinct key per workgroup instead of
    one per occurrence). Exact integer counts. torch.bincount off the GPU."""
    if keys.device.type != "cuda":
        return torch.bincount(keys.to(torch.int64), minlength=nbins)
    lib = require_game_lib()
    if keys.dtype not in (torch.int32, torch.int64):
        keys = keys.to(torch.int64)
    keys = keys.contiguous()
    counts = torch.zeros(max(int(nbins), 1), dtype=torch.int64, device=keys.device)
    if keys.numel():
        lo, hi = torch.aminmax(keys)
        if int(lo) < 0 or int(hi) >= nbins:
            raise ValueError(f"key_histogram: keys outside [0, {nbins})")
        check(lib.pml_key_hist(int(keys.dtype == torch.int32), keys.data_ptr(), keys.numel(), int(nbins),
                               counts.data_ptr(), stream_handle(keys.device)), "key_hist")
    return counts[:nbins]


def csr_gather_rows(nip: torch.Tensor, pos: torch.Tensor, val: torch.Tensor, rows: torch.Tensor, optr: torch.Tensor,
                    cbase: Optional[torch.Tensor] = None, col_dtype=torch.int64):
    """Rows ``rows`` of the CSR ``(nip, pos, val)`` (int64 / int64 / fp64) as a new CSR whose row r starts at
    ``optr[r]`` and spans ``optr[r + 1] - optr[r] >=`` its length slots (the rest zero: padding); columns minus
    ``cbase[r]`` when given, as ``col_dtype`` (int16 or int64). Returns ``(cols, vals)``
    (``csr_gather_rows_kernel``; torch off the GPU)."""
    nr = int(rows.numel())
    total = int(optr[-1]) if nr else 0
    dev = val.device
    assert col_dtype in (torch.int16, torch.int64) and optr.numel() == nr + 1
    ocol = torch.empty(total, dtype=col_dtype, device=dev)
    oval = torch.empty(total, dtype=torch.float64, device=dev)
    if nr == 0:
        return ocol, oval
    if dev.type != "cuda":
        lens = nip[rows + 1] - nip[rows]
        dl = optr[1:] - optr[:-1]
        r = torch.repeat_interleave(torch.arange(nr, device=dev), dl, output_size=total)
        t = torch.arange(total, device=dev) - optr[:-1][r]
        ok = t < lens[r]
        src = torch.where(ok, nip[rows][r] + t, torch.zeros_like(t))
        base = cbase[r] if cbase is not None else 0
        ocol.copy_(torch.where(ok, pos[src] - base, torch.zeros_like(t)).to(col_dtype))
        oval.copy_(torch.where(ok, val[src], torch.zeros((), dtype=torch.float64, device=dev)))
        return ocol, oval
    for t_ in (nip, pos, rows, optr) + (() if cbase is None else (cbase,)):
        assert t_.dtype == torch.int64 and t_.is_cuda and t_.is_contiguous()
    assert val.dtype == torch.float64 and val.is_contiguous()
    check(require_game_lib().pml_csr_gather_rows(
        int(col_dtype == torch.int16), nip.data_ptr(), pos.data_ptr(), val.data_ptr(), rows.data_ptr(), nr,
        optr.data_ptr(), None if cbase is None else cbase.data_ptr(), ocol.data_ptr(), oval.data_ptr(),
        stream_handle(dev)), "csr_gather_rows")
    return ocol, oval


def sorted_counts(sorted_keys: torch.Tensor, nbins: int) -> torch.Tensor:
    """Per-bin counts of NON-DECREASING keys in [0, nbins) (bincount without atomics: run boundaries by binary
    search)."""
    b = torch.searchsorted(sorted_keys, torch.arange(nbins + 1, device=sorted_keys.device, dtype=sorted_keys.dtype))
    return b[1:] - b[:-1]


def gemm_nt(A: torch.Tensor, Bm: torch.Tensor) -> torch.Tensor:
    """``A @ Bm.T`` for fp64 matrices (``gemm_nt_mfma_kernel``: fp64 MFMA, LDS-staged 32 x 32 tiles); torch
    off the GPU."""
    if A.device.type != "cuda" or A.dtype != torch.float64 or Bm.dtype != torch.float64:
        return A @ Bm.T
    lib = require_game_lib()
    A, Bm = A.contiguous(), Bm.contiguous()
    M, K = A.shape
    N, K2 = Bm.shape
    assert K == K2 and M < 2 ** 31 and N < 2 ** 31
    C = torch.empty(M, N, dtype=torch.float64, device=A.device)
    check(lib.pml_gemm_nt(M, N, K, A.data_ptr(), K, Bm.data_ptr(), K, C.data_ptr(), N, stream_handle(A.device)),
          "gemm_nt")
    return C


def spmm_rows(x, PT: torch.Tensor) -> torch.Tensor:
    """``X @ PT`` for a scipy CSR ``x`` [rows x D] and a dense fp64 device ``PT`` [D x k] (``spmm_rows_kernel``;
    the random projection's forward map)."""
    lib = require_game_lib()
    dev = PT.device
    x = x.tocsr()
    indptr = torch.from_numpy(x.indptr.astype("int64")).to(dev)
    col = torch.from_numpy(x.indices.astype("int32")).to(dev)
    val = torch.from_numpy(x.data.astype("float64")).to(dev)
    PT = PT.to(torch.float64).contiguous()
    n, k = x.shape[0], PT.shape[1]
    assert PT.shape[0] == x.shape[1]
    Y = torch.empty(n, k, dtype=torch.float64, device=dev)
    check(lib.pml_spmm_rows(indptr.data_ptr(), col.data_ptr(), val.data_ptr(), n, PT.data_ptr(), k, Y.data_ptr(),
                            stream_handle(dev)), "spmm_rows")
    return Y


SEG_GRAM_DMAX = 160 * 1024 // 8      # seg_gram_kernel's LDS image: one fp64 per projected column of the entity


def seg_gram(ents: torch.Tensor, n: int, row_ptr: torch.Tensor, col_ptr: torch.Tensor, nip: torch.Tensor,
             pos: torch.Tensor, val: torch.Tensor, dmax: Optional[int] = None,
             maxnnz: Optional[int] = None) -> torch.Tensor:
    """Per-entity Gram matrices ``K [B, n, n]`` (``seg_gram_kernel``) of the entities ``ents`` of a block-diagonal
    CSR (rows grouped by entity: ``row_ptr``; entity column ranges: ``col_ptr``; ``nip/pos/val`` = int64 indptr,
    int64 global columns, fp64 values, distinct columns per row). Entities with fewer than ``n`` rows are zero
    padded. Every entity needs ``d_e <= SEG_GRAM_DMAX`` (LDS image). Device only."""
    lib = require_game_lib()
    dev = ents.device
    B = int(ents.numel())
    K = torch.empty(B, n, n, dtype=torch.float64, device=dev)
    if B == 0:
        return K
    t = [x.to(dev).contiguous() for x in (ents, row_ptr, col_ptr, nip, pos)]
    for x in t[:4]:
        assert x.dtype == torch.int64
    assert t[4].dtype in (torch.int64, torch.int32)
    v = val.to(dev, torch.float64).contiguous()
    if dmax is None or maxnnz is None:
        # widest entity (LDS image) and most non-zeros of one entity (LDS staging of its entries): one readback
        e_lo, e_hi = row_ptr[ents], row_ptr[ents + 1]
        dmax, maxnnz = (int(x) for x in torch.stack([(col_ptr[ents + 1] - col_ptr[ents]).max(),
                                                      (nip[e_hi] - nip[e_lo]).max()]).tolist())
    if dmax > SEG_GRAM_DMAX:
        raise ValueError(f"seg_gram: an entity has {dmax} > {SEG_GRAM_DMAX} projected columns")
    stage = int(maxnnz) if os.environ.get("PML_SEG_GRAM_STAGE", "1") != "0" else 0
    check(lib.pml_seg_gram(B, n, dmax, stage, t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(),
                           t[4].data_ptr(), v.data_ptr(), K.data_ptr(), stream_handle(dev)), "seg_gram")
    return K


def batched_cholesky(K: torch.Tensor, nv: torch.Tensor):
    """In-place lower Cholesky factors of the fp64 batch ``K [B, n, n]`` (n <= 192; ``batched_chol_kernel``, one wave
    per problem, packed triangle in LDS); rows / columns ``>= nv[b]`` of problem b are treated as the identity.
    Returns ``(K, info)``: info[b] = 0, or the 1-based column of the first non-positive pivot (that factor is
    unusable, as with ``torch.linalg.cholesky_ex``)."""
    B, n, n2 = K.shape
    assert n == n2 and K.dtype == torch.float64 and K.is_contiguous()
    info = torch.zeros(B, dtype=torch.int32, device=K.device)
    if B == 0:
        return K, info
    if not K.is_cuda or n > 192:
        ar = torch.arange(n, device=K.device)
        pad = ar.unsqueeze(0) >= nv.to(K.device).unsqueeze(1)
        Kp = torch.where(pad.unsqueeze(1) | pad.unsqueeze(2), torch.zeros((), dtype=K.dtype, device=K.device), K)
        Kp = Kp + torch.diag_embed(pad.to(K.dtype))
        L, inf = torch.linalg.cholesky_ex(Kp)
        K.copy_(L)
        return K, inf.to(torch.int32)
    nv = nv.to(K.device, torch.int64).contiguous()
    check(require_game_lib().pml_batched_chol(B, n, nv.data_ptr(), K.data_ptr(), info.data_ptr(),
                                              stream_handle(K.device)), "batched_chol")
    return K, info


RS_PRIMAL_DMAX = 64 * 1024 // 8     # rs_primal_kernel: one fp64 LDS slot per projected column of the entity


def rs_primal(ents: torch.Tensor, row_ptr, col_ptr, nip, pos, val, r: torch.Tensor, W: torch.Tensor) -> None:
    """``W[col_ptr[e]:col_ptr[e+1]] = X_e^T r[rows of e]`` for the entities ``ents`` (int64) of a block-diagonal
    CSR (``nip``/``pos``/``val``: int64 indptr, int64 or int32 global columns, fp64 values; columns of an entity inside
    its ``col_ptr`` range, distinct inside a row) — ``rs_primal_kernel``, one wave per entity. In place on ``W``
    (fp64, packed like ``col_ptr``); every entity needs ``d_e <= RS_PRIMAL_DMAX``. Device only."""
    lib = require_game_lib()
    dev = W.device
    B = int(ents.numel())
    if B == 0:
        return
    t = [x.to(dev).contiguous() for x in (ents, row_ptr, col_ptr, nip, pos)]
    for x in t[:4]:
        assert x.dtype == torch.int64
    assert t[4].dtype in (torch.int64, torch.int32)
    v = val.to(dev, torch.float64).contiguous()
    assert r.dtype == torch.float64 and r.is_contiguous() and W.dtype == torch.float64 and W.is_contiguous()
    assert r.numel() >= int(row_ptr[-1]) and W.numel() >= int(col_ptr[-1])
    dmax = int((col_ptr[ents + 1] - col_ptr[ents]).max())
    if dmax > RS_PRIMAL_DMAX:
        raise ValueError(f"rs_primal: an entity has {dmax} > {RS_PRIMAL_DMAX} projected columns")
    check(lib.pml_rs_primal(B, dmax, t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(),
                            t[4].data_ptr(), v.data_ptr(), r.data_ptr(), W.data_ptr(), stream_handle(dev),
                            int(t[4].dtype == torch.int32)),
          "rs_primal")


def downsample_weights(y: torch.Tensor, w0: torch.Tensor, rate: float, binary: bool, seed: int,
                       rowid: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """K20 weight rewrite on the device (``downsample_kernel``); ``rowid`` = global row ids (int64) of the rows."""
    lib = require_game_lib()
    assert y.dtype == w0.dtype and y.dtype in (torch.float32, torch.float64) and y.numel() == w0.numel()
    out = torch.empty_like(w0) if out is None else out
    if rowid is not None:
        assert rowid.dtype == torch.int64 and rowid.numel() == y.numel() and rowid.device == y.device
    check(lib.pml_downsample(int(y.dtype == torch.float64), y.data_ptr(), w0.data_ptr(),
                             None if rowid is None else rowid.data_ptr(), y.numel(), seed & 0xFFFFFFFFFFFFFFFF,
                             float(rate), int(binary), out.data_ptr(), stream_handle(y.device)), "downsample")
    return out


_LDS_ORDER: dict = {}


def check_lds_add_order(device=None, trials: int = 512) -> dict:
    """Verify on ``device`` (once per process and device) the one ordering the bitwise determinism of the
    LDS-accumulating kernels rests on (glm_kernels.hip TL kernels, re_kernels.hip row passes): the lanes of one
    ds_add_f64 that hit the same address are applied in ascending lane order. ``trials`` waves add 64 values of
    spread magnitudes (the rounded sum depends on the order) into one LDS cell; the results are compared with the
    sequential lane-order sums and with a second run. Returns ``{"lane_order": bool, "repeatable": bool,
    "mismatches": int}``; ``PML_REQUIRE_DETERMINISM=1`` turns a failure into an error, otherwise it is logged
    once (results stay correct to rounding, but run-to-run bitwise equality is no longer guaranteed)."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if dev.type != "cuda":
        return {"skipped": "not a GPU device"}
    key = str(dev)
    if key in _LDS_ORDER:
        return _LDS_ORDER[key]
    lib = glm_lib()
    if lib is None:
        raise RuntimeError(f"native GLM kernel library missing ({lib_path('hip', 'glm')})")
    rng = np.random.default_rng(20261017)
    v = rng.standard_normal((trials, 64)) * np.exp2(rng.integers(-30, 31, (trials, 64)))
    ref = np.zeros(trials)
    for lane in range(64):                      # sequential, lane-ascending fp64 sums
        ref = ref + v[:, lane]
    vt = torch.from_numpy(v).to(dev)
    outs = []
    for _ in range(2):
        o = torch.empty(trials, dtype=torch.float64, device=dev)
        check(lib.pml_lds_add_order_probe(vt.data_ptr(), o.data_ptr(), int(trials), stream_handle(dev)),
              "lds_add_order_probe")
        outs.append(o.cpu().numpy())
    mism = int((outs[0] != ref).sum())
    res = {"lane_order": mism == 0, "repeatable": bool((outs[0] == outs[1]).all()), "mismatches": mism}
    _LDS_ORDER[key] = res
    if not (res["lane_order"] and res["repeatable"]):
        msg = (f"LDS same-address ds_add_f64 order check failed on {dev}: {res} — kernel results stay correct to "
               f"rounding, run-to-run bitwise equality is not guaranteed on this device")
        if os.environ.get("PML_REQUIRE_DETERMINISM", "0") == "1":
            raise RuntimeError(msg)
        import logging
        logging.getLogger(__name__).warning(msg)
    return res


def re_lib() -> Optional[ctypes.CDLL]:
    """Fused per-entity primal TRON (``ops/csrc/re_kernels.hip``)."""
    lib = _load("re")
    if lib is not None and not getattr(lib, "_pml_typed", False):
        lib.pml_re_tron_csr.argtypes = ([c_void_p, c_int] + [c_void_p] * 9 + [ctypes.c_longlong] + [c_void_p] * 6
                                        + [c_int, c_double, c_double, c_int, c_int, c_int, c_int, c_void_p])
        lib.pml_re_tron_csr.restype = c_int
        lib.pml_re_tron_smem.argtypes = [c_int]
        lib.pml_re_tron_smem.restype = ctypes.c_size_t
        lib.pml_re_tron_hess.argtypes = lib.pml_re_tron_csr.argtypes
        lib.pml_re_tron_lean.argtypes = lib.pml_re_tron_csr.argtypes[:-1] + [c_void_p, c_int, c_void_p, c_void_p]
        lib.pml_re_tron_lean.restype = c_int
        lib.pml_re_tron_hess.restype = c_int
        lib.pml_re_tron_hess_smem.argtypes = [c_int]
        lib.pml_re_tron_hess_smem.restype = ctypes.c_size_t
        lib.pml_re_tron_res.argtypes = ([c_void_p, c_void_p, c_int] + [c_void_p] * 4 + [c_int] + [c_void_p] * 14
                                        + [c_int, c_double, c_double, c_int, c_int, c_int, c_void_p])
        lib.pml_re_tron_res.restype = c_int
        lib.pml_rs_tron_big.argtypes = [c_int, c_int] + [c_void_p] * 9 + [c_int, c_double, c_double, c_int, c_int,
                                                                         c_int, c_void_p]
        lib.pml_rs_tron_big.restype = c_int
        lib.pml_re_res_cap.restype = c_int
        lib.pml_re_res_dmax.restype = c_int
        lib.pml_re_res_grid.restype = c_int
        lib.pml_re_res_ws_doubles.argtypes = [c_int]
        lib.pml_re_res_ws_doubles.restype = ctypes.c_size_t
        lib._pml_typed = True
    return lib


def require_re_lib() -> ctypes.CDLL:
    lib = re_lib()
    if lib is None:
        raise RuntimeError(
            f"native random-effect kernel library missing ({lib_path('hip', 're')}); run python -m photon_ml_amd.ops.build")
    return lib


# the lean streaming kernel takes launch classes up to this many coefficients (PML_RE_LEAN=0: never)
RE_LEAN_DMAX = 1024 if os.environ.get("PML_RE_LEAN", "1") != "0" else 0


def re_tron_csr(order, row_ptr, col_ptr, nip, lcol, val, y, off, wt, scr, W, f, iters, reason, zout, loss_id: int,
                l2: float, tol: float, max_iter: int, max_fail: int, max_cg: int, dmax: int,
                npass: Optional[torch.Tensor] = None, hessian: bool = False, gsc: Optional[torch.Tensor] = None,
                lean: Optional[bool] = None, quad: bool = False, xf2: Optional[torch.Tensor] = None) -> None:
    """Fused per-entity primal TRON over the entities ``order`` (int32; one workgroup each) of a block-diagonal
    CSR (``re_tron_csr_kernel``). Entity ``e`` owns rows ``row_ptr[e]:row_ptr[e+1]`` (int64) and coefficients
    ``col_ptr[e]:col_ptr[e+1]`` of the packed ``W`` (fp64, in: warm start, out: solution); ``nip`` int64 row
    pointers, ``lcol`` int16 entity-local columns (< d_e <= dmax, distinct inside a row), ``val`` fp64; ``y``,
    ``off``, ``wt`` per row; ``scr`` fp64 scratch of 4 x rows; outputs ``f`` / ``iters`` / ``reason`` per
    entity and ``zout`` (x_i . w per row); ``npass`` (optional int32 per entity): row passes run. ``hessian``:
    the tall-narrow kernel (``re_tron_hess_kernel``: d_e <= dmax <= 64, dmax a multiple of 16; the per-entity
    Hessian formed on the fp64 matrix cores, CG on it in LDS). ``lean`` (default: dmax <= 1024): the
    ``re_tron_lean_kernel`` (only the gathered vector + accumulators in LDS) with ``gsc`` (fp64 scratch like ``W``;
    allocated when None); ``quad``: every row of the batch is padded to whole quads of 4 entries (column 0, value
    0.0), and the lean kernel reads 4 columns / 4 values per lane load (row_pass_q). ``xf2`` (lean only, optional,
    fp64 per entity): ``||X_e||_F^2``; a warm start then scales its gradient tolerance by the bound
    ``||X_e||_F ||c||`` of ``||g(0)||`` and runs the pass at zero only if a gradient norm reaches it. Device only; in
    place, nothing returned."""
    lib = require_re_lib()
    n_rows = y.numel()
    B = int(order.numel())
    ts = (order, row_ptr, col_ptr, nip, lcol, val, y, off, wt, scr, W, f, iters, reason, zout)
    for t in ts:
        assert t.is_cuda and t.is_contiguous() and t.device == W.device
    assert order.dtype == torch.int32 and row_ptr.dtype == col_ptr.dtype == nip.dtype == torch.int64
    assert lcol.dtype == torch.int16 and nip.numel() == n_rows + 1 and lcol.numel() == val.numel()
    assert all(t.dtype == torch.float64 for t in (val, y, off, wt, scr, W, f, zout))
    assert off.numel() == n_rows and wt.numel() == n_rows and zout.numel() == n_rows and scr.numel() >= 4 * n_rows
    assert iters.dtype == reason.dtype == torch.int32
    if lean is None:
        lean = not hessian and dmax <= RE_LEAN_DMAX
    # lean launches size LDS to the launch's widest entity (a multiple of 8: four workgroups per CU up to 1008)
    assert (dmax % 16 == 0 and 16 <= dmax <= 64) if hessian else dmax % (8 if lean else 64) == 0
    n_ent = row_ptr.numel() - 1
    assert col_ptr.numel() == n_ent + 1 and f.numel() == n_ent
    if npass is not None:
        assert npass.is_cuda and npass.dtype == torch.int32 and npass.numel() == n_ent
    if os.environ.get("PML_CHECK_KERNEL_INPUTS", "0") == "1" and B:
        # the kernel indexes entities through ``order`` and sizes its LDS vectors by dmax
        assert int(order.min()) >= 0 and int(order.max()) < n_ent, "re_tron order out of range"
        oe = order.to(torch.int64)
        assert int((col_ptr[oe + 1] - col_ptr[oe]).max()) <= dmax, "entity wider than the launch's LDS class"
        assert W.numel() == int(col_ptr[-1]), "packed coefficients / column ranges inconsistent"
        nnz = int(nip[-1])
        assert int(row_ptr[-1]) == n_rows and nnz <= val.numel(), "row / non-zero ranges inconsistent"
        if lean and quad:
            # quad row pass (row_pass_q): every row starts on a quad and holds whole quads
            assert bool((nip % 4 == 0).all()), "quad lean kernel needs rows padded to multiples of 4 entries"
    args = [order.data_ptr(), B, row_ptr.data_ptr(), col_ptr.data_ptr(), nip.data_ptr(), lcol.data_ptr(),
            val.data_ptr(), y.data_ptr(), off.data_ptr(), wt.data_ptr(), scr.data_ptr(), n_rows, W.data_ptr(),
            f.data_ptr(), iters.data_ptr(), reason.data_ptr(), zout.data_ptr(),
            None if npass is None else npass.data_ptr(), int(loss_id), float(l2), float(tol), int(max_iter),
            int(max_fail), int(max_cg), int(dmax)]
    if lean:
        assert not hessian and dmax <= 1024
        if gsc is None:
            gsc = torch.empty_like(W)
        assert gsc.is_cuda and gsc.dtype == torch.float64 and gsc.numel() >= W.numel() and gsc.device == W.device
        if xf2 is not None:
            assert xf2.is_cuda and xf2.dtype == torch.float64 and xf2.numel() == n_ent and xf2.is_contiguous()
        check(lib.pml_re_tron_lean(*args, gsc.data_ptr(), int(bool(quad)), None if xf2 is None else xf2.data_ptr(),
                                   stream_handle(W.device)), "re_tron_lean")
        return
    fn = lib.pml_re_tron_hess if hessian else lib.pml_re_tron_csr
    check(fn(*args, stream_handle(W.device)), "re_tron_csr")


def re_res_params():
    """(rows per workgroup, max coefficients, resident workgroups on the current device) of the register-resident
    fused TRON (``re_tron_res_kernel``)."""
    lib = require_re_lib()
    return int(lib.pml_re_res_cap()), int(lib.pml_re_res_dmax()), int(lib.pml_re_res_grid())


def re_tron_res(task_ent, task_t0, ws, grid: int, row_ptr, col_ptr, nip, lcol, val, y, off, wt, W, f, iters, reason,
                zout, loss_id: int, l2: float, tol: float, max_iter: int, max_fail: int, max_cg: int,
                npass: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Register-resident fused per-entity primal TRON (``re_tron_res_kernel``): ONE persistent launch of ``grid``
    workgroups over the tasks ``task_ent`` (int32 entity per task, largest first) where task j is solved by the
    ``task_t0[j+1] - task_t0[j]`` workgroups of tickets ``task_t0[j] ..`` (a cluster when > 1; clusters first,
    ``ws`` holding 2 (dmax + 8) doubles per cluster ticket). Same data / outputs as :func:`re_tron_csr`. Returns
    the device error flag (int32[1]; non-zero = a cluster wait timed out and the results are invalid)."""
    lib = require_re_lib()
    n_rows = y.numel()
    n_tasks = int(task_ent.numel())
    dev = W.device
    for t in (task_ent, task_t0, ws, row_ptr, col_ptr, nip, lcol, val, y, off, wt, W, f, iters, reason, zout):
        assert t.is_cuda and t.is_contiguous() and t.device == dev
    assert task_ent.dtype == task_t0.dtype == torch.int32 and task_t0.numel() == n_tasks + 1
    assert row_ptr.dtype == col_ptr.dtype == nip.dtype == torch.int64 and lcol.dtype == torch.int16
    assert all(t.dtype == torch.float64 for t in (val, y, off, wt, W, f, zout, ws))
    assert nip.numel() == n_rows + 1 and off.numel() == n_rows and zout.numel() == n_rows
    cap, dmax, _ = re_res_params()
    if os.environ.get("PML_CHECK_KERNEL_INPUTS", "0") == "1" and n_tasks:
        te = task_ent.to(torch.int64)
        k = (task_t0[1:] - task_t0[:-1]).to(torch.int64)
        n_e = row_ptr[te + 1] - row_ptr[te]
        assert int(te.min()) >= 0 and int(te.max()) < row_ptr.numel() - 1, "task entity out of range"
        assert bool((k >= 1).all()) and int(k.max()) <= grid, "cluster larger than the resident grid"
        assert bool((n_e <= k * cap).all()) and bool((n_e > (k - 1) * cap).all()), "rows do not match members"
        assert int((col_ptr[te + 1] - col_ptr[te]).max()) <= dmax, "entity wider than the resident kernel"
        kk = k.tolist()
        cl = [i for i, v in enumerate(kk) if v > 1]
        assert cl == list(range(len(cl))), "cluster tasks must come first"
        need = int(task_t0[len(cl)]) if cl else 0
        assert ws.numel() >= need * 2 * (dmax + 8), "cluster workspace too small"
    ticket = torch.empty(1, dtype=torch.int32, device=dev)
    bar = torch.empty(max(n_tasks, 1), dtype=torch.int32, device=dev)
    err = torch.empty(1, dtype=torch.int32, device=dev)
    check(lib.pml_re_tron_res(task_ent.data_ptr(), task_t0.data_ptr(), n_tasks, ticket.data_ptr(), bar.data_ptr(),
                              ws.data_ptr(), err.data_ptr(), int(grid), row_ptr.data_ptr(), col_ptr.data_ptr(),
                              nip.data_ptr(), lcol.data_ptr(), val.data_ptr(), y.data_ptr(), off.data_ptr(),
                              wt.data_ptr(), W.data_ptr(), f.data_ptr(), iters.data_ptr(), reason.data_ptr(),
                              zout.data_ptr(), None if npass is None else npass.data_ptr(), int(loss_id), float(l2),
                              float(tol), int(max_iter), int(max_fail), int(max_cg), stream_handle(dev)),
          "re_tron_res")
    return err


def check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"{what} failed with HIP error {rc}")


def stream_handle(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream
