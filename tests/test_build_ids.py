"""Native libraries are tied to their sources by build ids (``photon_ml_amd/ops/build.py``): a library whose
stamp differs from the hash of the tree's sources is rebuilt or refused, never loaded (the reference ties its
artefacts to their sources through Gradle's incremental build, ``/root/reference/build.gradle:104-146``)."""
import shutil

import pytest

from photon_ml_amd.ops import build as B


def test_in_tree_libraries_carry_the_tree_build_ids():
    for kind, names in (("hip", B.HIP_SOURCES), ("cpp", B.CPP_SOURCES)):
        for name in names:
            path = B.lib_path(kind, name, False)
            if not path.exists():
                pytest.skip(f"{path} not built")
            assert B.read_stamp(path) == B.expected_id(kind, name, False), path


def test_build_id_covers_source_headers_and_flags(tmp_path):
    src = tmp_path / "k.cpp"
    src.write_text("int f() { return 1; }\n")
    a = B.build_id(src, ["-O3"])
    assert a == B.build_id(src, ["-O3"]) and len(a) == 16
    assert B.build_id(src, ["-O2"]) != a
    (tmp_path / "blocks.h").write_text("// header\n")
    assert B.build_id(src, ["-O3"]) != a


def test_loader_refuses_a_library_built_from_other_sources(tmp_path, monkeypatch):
    """Copy a source, build it, edit one byte: the old library is refused without a compiler and rebuilt with
    one; the rebuilt library carries the new id."""
    src = tmp_path / "csrc" / "index_map.cpp"
    src.parent.mkdir()
    shutil.copy(B.CPP_SOURCES["indexmap"], src)
    out = tmp_path / "_lib" / "libpml_indexmap.so"
    monkeypatch.setitem(B.CPP_SOURCES, "indexmap", src)
    monkeypatch.setattr(B, "lib_path", lambda kind, name, sanitize=None: out)
    B.compile_cpp(src, out, "indexmap")
    old_id = B.read_stamp(out)
    assert old_id == B.expected_id("cpp", "indexmap", False)
    assert B.verified_path("cpp", "indexmap", sanitize=False, auto_build=False) == out
    text = src.read_bytes()
    src.write_bytes(text.replace(b"return", b"return ", 1))          # one byte more in the source
    assert B.expected_id("cpp", "indexmap", False) != old_id
    with pytest.raises(B.StaleLibraryError):
        B.verified_path("cpp", "indexmap", sanitize=False, auto_build=False)
    monkeypatch.setenv("PML_NO_AUTOBUILD", "1")
    with pytest.raises(B.StaleLibraryError):
        B.verified_path("cpp", "indexmap", sanitize=False)
    monkeypatch.delenv("PML_NO_AUTOBUILD")
    assert B.verified_path("cpp", "indexmap", sanitize=False) == out        # rebuilt from the edited source
    assert B.read_stamp(out) == B.expected_id("cpp", "indexmap", False) != old_id


def test_stamp_is_read_without_loading(tmp_path):
    lib = tmp_path / "libx.so"
    lib.write_bytes(b"\x7fELF....PML_BUILD_ID=0123456789abcdef\0....")
    assert B.read_stamp(lib) == "0123456789abcdef"
    lib.write_bytes(b"\x7fELF no stamp")
    assert B.read_stamp(lib) is None
    assert B.read_stamp(tmp_path / "missing.so") is None
