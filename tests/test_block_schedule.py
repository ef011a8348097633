"""CPU tests of the HIP kernels' static block schedule (pml_build_blocks) via host emulation."""
import numpy as np
import pytest
import scipy.sparse as sp

from photon_ml_amd.ops import emulate


def _check(x: sp.csr_matrix, nb=None, maxseg=None):
    rng = np.random.default_rng(0)
    w = rng.normal(size=x.shape[1])
    out, blk = emulate.segment_sums(x.indptr.astype(np.int32), x.indices, x.data, w, nb, maxseg)
    np.testing.assert_allclose(out, x @ w, rtol=1e-12, atol=1e-12)
    xt = x.tocsc()
    r = rng.normal(size=x.shape[0])
    out_t, _ = emulate.segment_sums(xt.indptr.astype(np.int32), xt.indices, xt.data, r, nb, maxseg)
    np.testing.assert_allclose(out_t, x.T @ r, rtol=1e-12, atol=1e-12)
    out_sq, _ = emulate.segment_sums(xt.indptr.astype(np.int32), xt.indices, xt.data, r, nb, maxseg, square=True)
    np.testing.assert_allclose(out_sq, x.multiply(x).T @ r, rtol=1e-12, atol=1e-12)
    return blk


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_random_shapes(seed):
    rng = np.random.default_rng(seed)
    x = sp.random(700, 300, density=rng.uniform(0.001, 0.2), format="lil", random_state=seed)
    x[5, :] = 1.0  # long row relative to small nb
    x[:, 7] = 2.0  # long column
    x[9, :] = 0.0  # empty row
    _check(sp.csr_matrix(x), nb=64, maxseg=16)
    _check(sp.csr_matrix(x))


def test_empty_matrix():
    _check(sp.csr_matrix((10, 5)))


def test_exact_multiple_segments():
    x = sp.csr_matrix(np.ones((8, 64)))
    blk = _check(x, nb=64, maxseg=4)
    assert (blk[:, 4] == -1).all()
