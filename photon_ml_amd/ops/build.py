"""Build every native component in-tree (HIP kernels for gfx950 + host C++ runtime pieces).

* ``ops/csrc/*.hip``  -> ``ops/_lib/libpml_<name>.so`` via ``hipcc --offload-arch=gfx950 -O3 -shared -fPIC``
  (plain HIP, no hipify, no torch headers: the libraries expose a C ABI and are loaded with ctypes after torch
  so they share torch's HIP runtime — both resolve ``libamdhip64.so.7``).
* ``io/csrc/*.cpp``   -> ``io/_lib/libpml_<name>.so`` via ``g++ -O3 -shared -fPIC`` (Avro OCF codec, index map).

Run ``python -m photon_ml_amd.ops.build`` (or ``__graft_entry__.build()``).

**Build ids.** Every library is stamped with a content hash of what it was built from: the source, the headers
next to it, the compiler command line and the target arch (``build_id``). The hash is compiled in as
``-DPML_BUILD_ID=...`` — the C ABI libraries export it as ``pml_build_id()``, the pybind11 Avro module as
``build_id()``, and every library carries the marker string ``PML_BUILD_ID=<hash>`` that :func:`read_stamp` finds
without loading it. A library is rebuilt when its stamp differs from the hash of the tree's sources (not by
mtime), and the loaders refuse a library whose stamp does not match (:func:`verified_path`): a stale ``.so``
(the libraries are git-ignored and travel prebuilt) is rebuilt when a compiler is available and is otherwise an
error — it is never loaded. The reference ties its artefacts to their sources through Gradle's incremental build
(``/root/reference/build.gradle:104-146``).
"""
from __future__ import annotations

import hashlib
import os
import re
import shutil
import subprocess
import sys
from pathlib import Path
from typing import List, Optional

PKG = Path(__file__).resolve().parents[1]
HIP_SOURCES = {
    "glm": PKG / "ops" / "csrc" / "glm_kernels.hip",
    "game": PKG / "ops" / "csrc" / "game_kernels.hip",
    "re": PKG / "ops" / "csrc" / "re_kernels.hip",
}
CPP_SOURCES = {
    "avro": PKG / "io" / "csrc" / "avro_codec.cpp",
    "indexmap": PKG / "io" / "csrc" / "index_map.cpp",
}
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]
HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-Wno-unused-result"]
_STAMP_RE = re.compile(rb"PML_BUILD_ID=([0-9a-f]{16})")


class StaleLibraryError(RuntimeError):
    """A native library whose build id does not match the sources in the tree."""


def sanitize_enabled() -> bool:
    """``PML_NATIVE_SANITIZE=1``: load the AddressSanitizer + UBSan builds of the HOST C++ libraries (Avro codec,
    index map). GPU sanitizers are unavailable on the target pool, so device code is checked by host-side shape
    validation and the kernel parity tests instead (SURVEY §5 race detection / sanitizers)."""
    return os.environ.get("PML_NATIVE_SANITIZE", "0") == "1"


def lib_path(kind: str, name: str, sanitize: bool = None) -> Path:
    base = PKG / ("ops" if kind == "hip" else "io") / "_lib"
    if sanitize is None:
        sanitize = kind != "hip" and sanitize_enabled()
    return base / f"libpml_{name}{'_asan' if sanitize else ''}.so"


def _deps(src: Path) -> List[Path]:
    """The source and the headers next to it (e.g. generated asm blocks)."""
    return [src] + sorted(src.parent.glob("*.h"))


def build_id(src: Path, flags: List[str]) -> str:
    """16-hex-digit content hash of ``src``, its sibling headers and the compile command (flags + arch)."""
    h = hashlib.sha256()
    for d in _deps(src):
        h.update(d.name.encode() + b"\0" + d.read_bytes() + b"\0")
    h.update("\0".join(flags).encode())
    return h.hexdigest()[:16]


def read_stamp(lib: Path) -> Optional[str]:
    """The build id a library was stamped with (None: missing file or no stamp)."""
    try:
        m = _STAMP_RE.search(Path(lib).read_bytes())
    except OSError:
        return None
    return m.group(1).decode() if m else None


def _hipcc() -> str:
    for c in ("hipcc", "/opt/rocm/bin/hipcc"):
        if shutil.which(c):
            return shutil.which(c)
    raise RuntimeError("hipcc not found")


def _hip_flags(extra: List[str] = ()) -> List[str]:
    return [f"--offload-arch={ARCH}", *HIP_FLAGS, *extra]


def _cpp_flags(name: str, sanitize: bool) -> List[str]:
    vis = ["-fvisibility=hidden"] if name == "avro" else []  # pybind11 module vs plain C ABI
    opt = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined"] if sanitize else ["-O3"]
    return [*opt, "-std=c++17", "-fPIC", "-shared", "-pthread", *vis]


def expected_id(kind: str, name: str, sanitize: bool = None) -> str:
    """Build id the tree's sources give the library ``kind`` ('hip' / 'cpp') ``name``."""
    if kind == "hip":
        return build_id(HIP_SOURCES[name], _hip_flags())
    sanitize = sanitize_enabled() if sanitize is None else sanitize
    return build_id(CPP_SOURCES[name], _cpp_flags(name, sanitize))


def _compile(cmd_of, out: Path, bid: str, force: bool, verbose: bool) -> None:
    """Build ``out`` (stamped ``bid``) unless it already carries that stamp. Concurrent builders (torchrun ranks,
    xdist workers that all find the library stale) serialise on an ``fcntl`` lock next to the library and re-check
    the stamp once they hold it; each compiles into its own temporary file, replaced atomically."""
    import fcntl
    if not force and read_stamp(out) == bid:
        return
    out.parent.mkdir(parents=True, exist_ok=True)
    with open(str(out) + ".lock", "a+") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            if not force and read_stamp(out) == bid:       # another process built it while we waited
                return
            tmp = f"{out}.{os.getpid()}.tmp"
            cmd = cmd_of(tmp)
            if verbose:
                print(" ".join(cmd), flush=True)
            try:
                subprocess.run(cmd, check=True)
                os.replace(tmp, out)
            finally:
                if os.path.exists(tmp):
                    os.unlink(tmp)
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)


def compile_hip(src: Path, out: Path, extra: List[str] = (), force: bool = False, verbose: bool = False) -> Path:
    """hipcc ``src`` into ``out`` stamped with its build id; skipped when ``out`` already carries that id."""
    flags = _hip_flags(extra)
    bid = build_id(src, flags)
    _compile(lambda tmp: [_hipcc(), *flags, f'-DPML_BUILD_ID="{bid}"', str(src), "-o", tmp], out, bid, force,
             verbose)
    return out


def compile_cpp(src: Path, out: Path, name: str, sanitize: bool = False, force: bool = False,
                verbose: bool = False) -> Path:
    flags = _cpp_flags(name, sanitize)
    bid = build_id(src, flags)

    def cmd(tmp):
        import sysconfig
        import pybind11
        inc = ["-I" + sysconfig.get_paths()["include"], "-I" + pybind11.get_include()]
        return ["g++", *flags, f'-DPML_BUILD_ID="{bid}"', *inc, str(src), "-o", tmp, "-lz"]
    _compile(cmd, out, bid, force, verbose)
    return out


def build_hip(name: str, force: bool = False, verbose: bool = False) -> Path:
    src = HIP_SOURCES[name]
    out = lib_path("hip", name)
    if not src.exists():
        return out
    return compile_hip(src, out, force=force, verbose=verbose)


def build_experiment(force: bool = False, verbose: bool = False) -> Path:
    """Profiling build of the GLM kernels with the runtime ablation switches compiled in (``-DPML_TL_EXPERIMENT``,
    ``libpml_glm_abl.so``; load it with ``PML_GLM_LIB=<path>``). Never used in production."""
    return compile_hip(HIP_SOURCES["glm"], lib_path("hip", "glm_abl"), ["-DPML_TL_EXPERIMENT"], force, verbose)


def build_cpp(name: str, force: bool = False, verbose: bool = False, sanitize: bool = None) -> Path:
    src = CPP_SOURCES[name]
    sanitize = sanitize_enabled() if sanitize is None else sanitize
    out = lib_path("cpp", name, sanitize)
    if not src.exists():
        return out
    return compile_cpp(src, out, name, sanitize, force, verbose)


def _have_compiler(kind: str) -> bool:
    if kind == "hip":
        return any(shutil.which(c) for c in ("hipcc", "/opt/rocm/bin/hipcc"))
    return shutil.which("g++") is not None


def verify_stamp(lib: Path, expected: str, what: str) -> None:
    """Raise :class:`StaleLibraryError` unless ``lib`` carries build id ``expected``."""
    got = read_stamp(lib)
    if got != expected:
        raise StaleLibraryError(
            f"{what}: {lib} was built from other sources (build id {got}, the tree's sources give {expected}); "
            f"rebuild it with python -m photon_ml_amd.ops.build")


def verified_path(kind: str, name: str, sanitize: bool = None, auto_build: bool = True) -> Path:
    """Path of an up-to-date library ``kind``/``name``: (re)built when missing or stale if a compiler is available
    (and ``PML_NO_AUTOBUILD`` is not 1), else :class:`StaleLibraryError` / FileNotFoundError — a library whose
    stamp does not match the tree's sources is never handed to a loader."""
    if kind == "cpp" and sanitize is None:
        sanitize = sanitize_enabled()
    path = lib_path(kind, name, sanitize)
    want = expected_id(kind, name, sanitize)
    if read_stamp(path) != want and auto_build and os.environ.get("PML_NO_AUTOBUILD") != "1" \
            and _have_compiler(kind):
        if kind == "hip":
            build_hip(name)
        else:
            build_cpp(name, sanitize=sanitize)
    if not path.exists():
        raise FileNotFoundError(f"native library {path} missing; run python -m photon_ml_amd.ops.build")
    verify_stamp(path, want, f"native library {name}")
    return path


def build_all(force: bool = False, verbose: bool = False):
    """Build every library whose stamp is out of date, the compiler processes in parallel."""
    from concurrent.futures import ThreadPoolExecutor
    jobs = [(build_hip, n) for n, src in HIP_SOURCES.items() if src.exists()]
    jobs += [(build_cpp, n) for n, src in CPP_SOURCES.items() if src.exists()]
    with ThreadPoolExecutor(max_workers=min(len(jobs), max(1, (os.cpu_count() or 1) // 2), 5)) as ex:
        futs = [ex.submit(fn, n, force, verbose) for fn, n in jobs]
        return [f.result() for f in futs]


if __name__ == "__main__":
    for p in build_all(force="--force" in sys.argv, verbose=True):
        print(p, p.exists(), read_stamp(p))
