"""The CI gate's fail-on-skip policy (tests/conftest.py, scripts/ci.sh; the reference's FailOnSkipListener): with
PML_FAIL_ON_SKIP=1 a skip outside tests/skip_allowlist.txt fails, an allowlisted one does not, and without the
variable skips stay skips."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def _run(tmp_path, body, fail_on_skip):
    d = tmp_path / "tests"
    d.mkdir(exist_ok=True)
    (d / "conftest.py").write_text(open(os.path.join(HERE, "conftest.py")).read())
    (d / "skip_allowlist.txt").write_text("test_allowed.py :: fixture absent\n")
    for name, src in body.items():
        (d / name).write_text(src)
    env = dict(os.environ, PML_FAIL_ON_SKIP="1" if fail_on_skip else "0")
    return subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider", str(d)], cwd=tmp_path,
                          env=env, capture_output=True, text=True, timeout=300)


SKIPPING = "import pytest\ndef test_x():\n    pytest.skip('something missing')\n"
ALLOWED = "import pytest\n@pytest.mark.skipif(True, reason='fixture absent')\ndef test_y():\n    pass\n"


def test_unlisted_skip_fails_under_the_gate(tmp_path):
    r = _run(tmp_path, {"test_skipping.py": SKIPPING}, True)
    assert r.returncode != 0 and "skip_allowlist" in r.stdout, r.stdout[-2000:]


def test_allowlisted_skip_passes_under_the_gate(tmp_path):
    r = _run(tmp_path, {"test_allowed.py": ALLOWED}, True)
    assert r.returncode == 0 and "1 skipped" in r.stdout, r.stdout[-2000:]


def test_skips_stay_skips_without_the_gate(tmp_path):
    r = _run(tmp_path, {"test_skipping.py": SKIPPING}, False)
    assert r.returncode == 0 and "1 skipped" in r.stdout, r.stdout[-2000:]


def test_experiment_variants_are_deselected_not_skipped(tmp_path):
    src = "import pytest\n@pytest.mark.experiment\ndef test_variant():\n    pass\ndef test_prod():\n    pass\n"
    r = _run(tmp_path, {"test_exp.py": src}, True)
    assert r.returncode == 0 and "1 passed" in r.stdout and "1 deselected" in r.stdout, r.stdout[-2000:]
