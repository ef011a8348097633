"""Host C++ runtime under AddressSanitizer + UBSan (SURVEY §5 "race detection / sanitizers").

The Avro OCF codec (deflate / snappy / null, columnar reader) and the mmap index map are rebuilt with
``-fsanitize=address,undefined`` (``PML_NATIVE_SANITIZE=1`` selects the ``*_asan.so`` builds) and exercised in a
child interpreter with the sanitizer runtimes preloaded; any heap overflow, use-after-free or UB aborts the
child. GPU sanitizers are not available on the target pool; device kernels are covered by host-side shape
validation and the kernel parity tests.
"""
import os
import shutil
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _runtime(name):
    p = subprocess.run(["g++", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.mark.skipif(shutil.which("g++") is None or _runtime("libasan.so") is None, reason="no g++/ASan runtime")
def test_native_io_under_asan_ubsan(tmp_path):
    sys.path.insert(0, ROOT)
    from photon_ml_amd.ops.build import build_cpp
    for n in ("avro", "indexmap"):
        build_cpp(n, sanitize=True)
    code = textwrap.dedent(f"""
        import os, sys, random
        sys.path.insert(0, {ROOT!r})
        from photon_ml_amd.io import avro
        from photon_ml_amd.io.index_map import build_offheap_index_map
        assert avro.native().__file__.endswith("_asan.so"), avro.native().__file__
        rnd = random.Random(0)
        recs = []
        for i in range(3000):
            feats = [{{"name": "f%d" % rnd.randrange(500), "term": rnd.choice(["", "t1", "t\\u00e9"]),
                      "value": rnd.uniform(-5, 5)}} for _ in range(rnd.randrange(0, 12))]
            recs.append({{"label": float(i % 2), "features": feats, "weight": 1.0 if i % 3 else None,
                         "offset": 0.5, "uid": str(i), "metadataMap": {{"userId": "u%d" % (i % 37)}}}})
        for codec in ("null", "deflate", "snappy"):
            p = os.path.join({str(tmp_path)!r}, codec + ".avro")
            avro.write_records(p, avro.TRAINING_EXAMPLE, recs, codec=codec, block_records=257)
            back = avro.read_records(p)[1]
            assert len(back) == len(recs) and back[17]["features"] == recs[17]["features"], codec
        assert avro.native().snappy_roundtrip("x" * 100000 + "abc" * 777)
        keys = ["f%d\\u0001t%d" % (i, i % 3) for i in range(2000)]
        im = build_offheap_index_map(keys, os.path.join({str(tmp_path)!r}, "im"), "global", n_partitions=3)
        assert len(set(im.get_index(k) for k in keys)) == len(keys)
        assert im.get_index("missing\\u0001") in (-1, None)
        print("SANITIZED OK")
    """)
    env = dict(os.environ, PML_NATIVE_SANITIZE="1",
               LD_PRELOAD=" ".join(p for p in (_runtime("libasan.so"), _runtime("libubsan.so")) if p),
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:symbolize=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0 and "SANITIZED OK" in r.stdout, (r.stdout[-2000:], r.stderr[-6000:])
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-6000:]
