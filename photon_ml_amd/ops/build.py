"""Build every native component in-tree (HIP kernels for gfx950 + host C++ runtime pieces).

* ``ops/csrc/*.hip``  -> ``ops/_lib/libpml_<name>.so`` via ``hipcc --offload-arch=gfx950 -O3 -shared -fPIC``
  (plain HIP, no hipify, no torch headers: the libraries expose a C ABI and are loaded with ctypes after torch
  so they share torch's HIP runtime — both resolve ``libamdhip64.so.7``).
* ``io/csrc/*.cpp``   -> ``io/_lib/libpml_<name>.so`` via ``g++ -O3 -shared -fPIC`` (Avro OCF codec, index map).

Run ``python -m photon_ml_amd.ops.build`` (or ``__graft_entry__.build()``). Rebuilds only when sources are newer.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

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


def _needs_build(src: Path, out: Path) -> bool:
    """Out of date when the source or any header next to it (e.g. generated asm blocks) is newer."""
    if not out.exists():
        return True
    deps = [src] + sorted(src.parent.glob("*.h"))
    return max(d.stat().st_mtime for d in deps) > out.stat().st_mtime


def _hipcc() -> str:
    for c in ("hipcc", "/opt/rocm/bin/hipcc"):
        if shutil.which(c):
            return shutil.which(c)
    raise RuntimeError("hipcc not found")


def build_hip(name: str, force: bool = False, verbose: bool = False) -> Path:
    src = HIP_SOURCES[name]
    out = lib_path("hip", name)
    if not src.exists():
        return out
    out.parent.mkdir(parents=True, exist_ok=True)
    if force or _needs_build(src, out):
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-Wno-unused-result", str(src), "-o", str(out) + ".tmp"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(str(out) + ".tmp", out)
    return out


def build_experiment(force: bool = False, verbose: bool = False) -> Path:
    """Profiling build of the GLM kernels with the runtime ablation switches compiled in (``-DPML_TL_EXPERIMENT``,
    ``libpml_glm_abl.so``; load it with ``PML_GLM_LIB=<path>``). Never used in production."""
    src = HIP_SOURCES["glm"]
    out = lib_path("hip", "glm_abl")
    out.parent.mkdir(parents=True, exist_ok=True)
    if force or _needs_build(src, out):
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-DPML_TL_EXPERIMENT",
               "-Wno-unused-result", str(src), "-o", str(out) + ".tmp"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(str(out) + ".tmp", out)
    return out


def build_cpp(name: str, force: bool = False, verbose: bool = False, sanitize: bool = None) -> Path:
    src = CPP_SOURCES[name]
    sanitize = sanitize_enabled() if sanitize is None else sanitize
    out = lib_path("cpp", name, sanitize)
    if not src.exists():
        return out
    out.parent.mkdir(parents=True, exist_ok=True)
    if force or _needs_build(src, out):
        import sysconfig
        import pybind11
        inc = ["-I" + sysconfig.get_paths()["include"], "-I" + pybind11.get_include()]
        vis = ["-fvisibility=hidden"] if name == "avro" else []  # pybind11 module vs plain C ABI
        opt = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
               "-fno-sanitize-recover=undefined"] if sanitize else ["-O3"]
        cmd = ["g++", *opt, "-std=c++17", "-fPIC", "-shared", "-pthread", *vis, *inc, str(src), "-o",
               str(out) + ".tmp", "-lz"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(str(out) + ".tmp", out)
    return out


def build_all(force: bool = False, verbose: bool = False):
    outs = []
    for n, src in HIP_SOURCES.items():
        if src.exists():
            outs.append(build_hip(n, force, verbose))
    for n, src in CPP_SOURCES.items():
        if src.exists():
            outs.append(build_cpp(n, force, verbose))
    return outs


if __name__ == "__main__":
    for p in build_all(force="--force" in sys.argv, verbose=True):
        print(p, p.exists())
