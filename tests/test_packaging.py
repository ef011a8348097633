"""Installable distribution (the reference's module jars + shaded photon-all jar launched with spark-submit,
/root/reference/photon-all/build.gradle:20-101): ``pip install .`` into a scratch virtual environment (offline:
no build isolation) installs the package with its stamped native libraries and the driver launchers."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.slow
def test_pip_install_into_scratch_venv_gives_working_launchers(tmp_path):
    venv = tmp_path / "venv"
    # no ensurepip in the image: the venv sees the system site-packages (torch, pip, setuptools)
    subprocess.run([sys.executable, "-m", "venv", "--without-pip", "--system-site-packages", str(venv)], check=True)
    py = venv / "bin" / "python"
    env = dict(os.environ, PIP_NO_CACHE_DIR="1", PIP_DISABLE_PIP_VERSION_CHECK="1")
    env.pop("PYTHONPATH", None)
    p = subprocess.run([str(py), "-m", "pip", "install", "--no-build-isolation", "--no-deps", "-q", REPO],
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=1200)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    site = subprocess.run([str(py), "-c", "import photon_ml_amd, os; print(os.path.dirname(photon_ml_amd.__file__))"],
                          cwd=tmp_path, env=env, capture_output=True, text=True, check=True).stdout.strip()
    assert site.startswith(str(venv)), site                    # the installed copy, not the checkout
    for lib in ("ops/_lib/libpml_glm.so", "ops/_lib/libpml_re.so", "ops/_lib/libpml_game.so",
                "io/_lib/libpml_avro.so", "io/_lib/libpml_indexmap.so", "ops/csrc/glm_kernels.hip"):
        assert os.path.exists(os.path.join(site, lib)), lib
    for cmd, flag in (("game-training", "--coordinate-configurations"), ("game-scoring", "--model-input-directory"),
                      ("photon-ml", "--training-data-directory"), ("feature-indexing", "--num-storage-partitions"),
                      ("feature-bags", "--feature-bags-keys"), ("libsvm-to-avro", "usage")):
        r = subprocess.run([str(venv / "bin" / cmd), "--help"], cwd=tmp_path, env=env, capture_output=True,
                           text=True, timeout=300)
        assert r.returncode == 0 and flag in r.stdout, (cmd, r.stdout[-2000:], r.stderr[-2000:])
    # the installed host libraries load and carry the build ids of the installed sources
    r = subprocess.run([str(py), "-c", "from photon_ml_amd.io import avro; from photon_ml_amd.ops.build import "
                        "expected_id; assert avro.native().build_id() == expected_id('cpp', 'avro'); print('ok')"],
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]
