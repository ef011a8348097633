"""Tiled (TL) layout construction on the CPU: packing, block/item tables and a host emulation of the kernels'
arithmetic against scipy (the GPU kernels are checked against the same reference in test_kernels_gpu.py)."""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from photon_ml_amd.ops.tiled import TLFwdChunk, TLTChunk, fwd_bits, t_bits, tl_supported


@pytest.mark.parametrize("il", [0, 1])
@pytest.mark.parametrize("m,d,dens,item", [(3000, 500, 0.05, 64), (5000, 70000, 0.0005, 1 << 16), (100, 7, 0.5, 8),
                                           (2048, 4096, 0.01, 300), (10, 3, 0.0, 64)])
def test_tl_emulation_matches_scipy(m, d, dens, item, il):
    rng = np.random.default_rng(0)
    x = sp.random(m, d, density=dens, format="csr", random_state=1)
    x.data = rng.normal(size=x.nnz)
    rp = torch.from_numpy(x.indptr.astype(np.int64))
    col = torch.from_numpy(x.indices.astype(np.int64))
    val = torch.from_numpy(x.data)
    f = TLFwdChunk(rp, col, val, d, il=il)
    t = TLTChunk(rp, col, val, d, m, item_entries=item, il=il)
    w = rng.normal(size=d)
    r = rng.normal(size=m)
    np.testing.assert_allclose(f.emulate_matvec(torch.from_numpy(w)).numpy(), x @ w, atol=1e-12)
    np.testing.assert_allclose(t.emulate_rmatvec(torch.from_numpy(r)).numpy(), x.T @ r, atol=1e-12)
    np.testing.assert_allclose(t.emulate_rmatvec(torch.from_numpy(r), square=True).numpy(),
                               x.multiply(x).T @ r, atol=1e-12)
    # tables: blocks cover rows in order, items cover every entry exactly once, tile by tile
    b = f.blk.numpy()
    assert b[0, 0] == 0 and (b[1:, 0] == b[:-1, 0] + b[:-1, 1]).all() and b[-1, 0] + b[-1, 1] == m
    it = t.items.numpy()
    if len(it):
        cnt = t.unit_counts().numpy()
        assert it[0, 1] == 0 and (cnt <= item).all() and cnt.sum() == x.nnz
        if il:  # round-aligned, zero-padded windows
            assert (it[:, 1] % 256 == 0).all() and (it[1:, 1] >= it[:-1, 2]).all()
            assert (b[:, 2] % 256 == 0).all()
        else:
            assert (it[1:, 1] == it[:-1, 2]).all() and it[-1, 2] == x.nnz
        assert t.nparts == int((it[:, 3] >= 0).sum())
    # forward blocks: entries sorted by column inside a block (in logical order)
    pk, _ = f.logical()
    p = pk.to(torch.int64).numpy() & 0xFFFFFFFF
    # forward blocks: narrow section then wide section, each sorted by column (in logical order)
    nn = 256 * (b[:, 5] - b[:, 4])
    starts = np.r_[0, np.cumsum(f.unit_counts().numpy())]
    for lo, hi, k in zip(starts[:-1], starts[1:], nn):
        for a, z in ((lo, lo + k), (lo + k, hi)):
            assert (np.diff(p[a:z] >> f.rbits) >= 0).all()
    if il and x.nnz:
        # lane L's quad of a round holds logical entries L, L+64, L+128, L+192 of that round
        lo = int(b[0, 2])
        n0 = int(b[0, 3] - b[0, 2])
        if n0 >= 256 and b[0, 5] == b[0, 4]:
            phys = f.pack[lo:lo + 256].to(torch.int64).numpy()
            logi = p[:256].astype(np.int64)
            phys_u = phys & 0xFFFFFFFF
            assert (phys_u.reshape(64, 4).T.reshape(-1) == logi).all()


def test_bits():
    assert fwd_bits(1_000_000) == 10 and t_bits(1 << 20) == 10 and fwd_bits(1_000_000, want=12) == 12
    assert fwd_bits(1 << 26) == 6 and fwd_bits(1 << 28) is None and t_bits(1 << 20, f64=True, want=12) == 11
    assert not tl_supported(1 << 28, 1 << 20) and tl_supported(1 << 24, 1 << 22)


@pytest.mark.parametrize("layout", ["tiled", "segmented"])
def test_device_data_construction_cpu(layout):
    """DeviceGLMData tables/scratch sizing for both layouts (construction only: kernels need a GPU)."""
    from photon_ml_amd.data.synthetic import generate_glm_data
    from photon_ml_amd.ops.device import DeviceGLMData
    data, _ = generate_glm_data("LOGISTIC_REGRESSION", 3000, 300, density=0.05, seed=2)
    dev = DeviceGLMData.from_labeled(data, "cpu", "bf16", chunk_rows=1000, layout=layout, item_entries=500)
    assert dev.layout == layout and len(dev.csr) == 3 and len(dev.csc) == 3
    assert dev.stats.numel() >= 2 * sum(c.nstats for c in dev.csr)
    assert dev.parts.numel() >= max(c.parts_needed for c in dev.csc)
    if layout == "tiled":
        assert dev.validate()
        # a corrupted gather index is caught on the host before any kernel could read out of bounds
        f = dev.csr[1]
        lo = int(f.blk[0, 2])
        f.pack[lo] = (300 + 5) << f.rbits
        with pytest.raises(ValueError, match="gather index"):
            dev.validate()


@pytest.mark.parametrize("chunk,item,hot", [(700, 64, False), (1000, 300, True), (5000, 1 << 16, False)])
def test_tl_shard_wide_transpose_emulation(chunk, item, hot):
    """Shard-wide transpose tables (all chunks in one launch): every entry once, split tiles combined in
    (chunk, item) order, single-item tiles direct; result == X^T r."""
    from photon_ml_amd.ops.tiled import TLTMulti, combine_seg
    rng = np.random.default_rng(3)
    m, d = 5000, 3000
    x = sp.random(m, d, density=0.01, format="lil", random_state=2)
    if hot:
        x[:, 5] = 1.0  # a column in every row -> tiles with many items across chunks
    x = x.tocsr()
    x.data = rng.normal(size=x.nnz)
    starts = list(range(0, m, chunk)) + [m]
    chunks = []
    for a, b in zip(starts[:-1], starts[1:]):
        xc = x[a:b]
        chunks.append(TLTChunk(torch.from_numpy(xc.indptr.astype(np.int64)),
                               torch.from_numpy(xc.indices.astype(np.int64)), torch.from_numpy(xc.data), d, chunk,
                               item_entries=item))
    mt = TLTMulti(chunks, starts, d)
    r = rng.normal(size=m)
    np.testing.assert_allclose(mt.emulate_rmatvec(torch.from_numpy(r)).numpy(), x.T @ r, atol=1e-11)
    np.testing.assert_allclose(mt.emulate_rmatvec(torch.from_numpy(r), square=True).numpy(),
                               x.multiply(x).T @ r, atol=1e-11)
    it = mt.items.numpy()
    assert it.shape == (sum(c.nitems for c in chunks), 8)
    assert mt.nparts == int((it[:, 4] >= 0).sum()) and sorted(it[it[:, 4] >= 0, 4]) == list(range(mt.nparts))
    # a tile is direct iff it has exactly one item in the shard
    tiles, cnt = np.unique(it[:, 1], return_counts=True)
    single = set(tiles[cnt == 1].tolist())
    assert all((row[4] < 0) == (row[1] in single) for row in it)
    cu = mt.cu.numpy()[: mt.ncu]
    k_of_unit = np.bincount(it[it[:, 4] >= 0, 1])[mt.mt_tiles.numpy()[cu[:, 0]]]
    assert (cu[:, 2] - cu[:, 1] <= np.array([combine_seg(int(k)) for k in k_of_unit])).all()
    assert mt.mt_ptr.numpy()[-1] == mt.ncu
    # re-streaming over copies of the same units (row-sampled shards) keeps every table but the stream windows
    import copy as _copy
    moved = []
    for ch in chunks:
        cc = _copy.copy(ch)
        cc.items = ch.items.clone()
        cc.items[:, 1] += 256          # shifted windows, as a compacted stream would have
        cc.items[:, 2] += 256
        moved.append(cc)
    rt = mt.restreamed(moved)
    rit = rt.items.numpy()
    assert np.array_equal(rit[:, [0, 1, 4, 5, 6, 7]], it[:, [0, 1, 4, 5, 6, 7]])
    assert np.array_equal(rit[:, 2:4], it[:, 2:4] + 256)
    for tile_range in ((0, 1), (1, 3)):
        bt = TLTMulti(chunks, starts, d, tile_range=tile_range)
        bit = bt.restreamed(moved).items.numpy()
        assert np.array_equal(bit[:, 2:4], bt.items.numpy()[:, 2:4] + 256)


@pytest.mark.parametrize("il", [0, 1])
def test_feature_statistics_from_device_shard_match_host(il, monkeypatch):
    """BasicStatisticalSummary.from_device (column reductions over the tiled streams, relabelling undone) ==
    the host scipy computation (MLlib colStats semantics, implicit zeros in max/min)."""
    from photon_ml_amd.data.synthetic import generate_glm_data
    from photon_ml_amd.ops import tiled
    from photon_ml_amd.ops.device import DeviceGLMData
    from photon_ml_amd.stat.summary import BasicStatisticalSummary
    monkeypatch.setattr(tiled, "INTERLEAVE", il)
    data, _ = generate_glm_data("LOGISTIC_REGRESSION", 3000, 200, density=0.05, seed=4)
    dev = DeviceGLMData.from_labeled(data, "cpu", "f64", chunk_rows=1000, layout="tiled", relabel=True)
    a = BasicStatisticalSummary.from_device(dev)
    b = BasicStatisticalSummary.compute(data.x)
    for f in ("mean", "variance", "num_nonzeros", "max", "min", "norm_l1", "norm_l2", "mean_abs"):
        np.testing.assert_allclose(getattr(a, f).numpy(), getattr(b, f).numpy(), rtol=1e-12, atol=1e-12, err_msg=f)
    assert a.count == b.count


def test_narrow_rounds_on_zipf_data_cpu():
    """Zipf columns (bench-like): a large share of entries lands in narrow rounds in both copies; the emulated
    products still equal scipy and every narrow key window lies inside the gathered vector."""
    from photon_ml_amd.ops.tiled import NARROW_W
    rng = np.random.default_rng(5)
    m, d, k = 6000, 5000, 12
    ranks = np.minimum(rng.zipf(1.3, size=(m, k)) - 1, d - 1)
    rows = np.repeat(np.arange(m), k)
    x = sp.csr_matrix((rng.normal(size=m * k), (rows, ranks.ravel())), shape=(m, d))
    x.sum_duplicates()
    rp = torch.from_numpy(x.indptr.astype(np.int64))
    col = torch.from_numpy(x.indices.astype(np.int64))
    val = torch.from_numpy(x.data)
    f = TLFwdChunk(rp, col, val, d, il=1)
    t = TLTChunk(rp, col, val, d, m, item_entries=1 << 14, il=1)
    for ch, n in ((f, x.nnz), (t, x.nnz)):
        assert ch.n_narrow_rounds * 256 > 0.2 * n
        assert int(ch.nbase.min()) >= 0
    assert int(f.nbase.max()) + NARROW_W <= d and int(t.nbase.max()) + NARROW_W <= m
    w, r = rng.normal(size=d), rng.normal(size=m)
    np.testing.assert_allclose(f.emulate_matvec(torch.from_numpy(w)).numpy(), x @ w, atol=1e-11)
    np.testing.assert_allclose(t.emulate_rmatvec(torch.from_numpy(r)).numpy(), x.T @ r, atol=1e-11)


def test_wide_round_bases_keep_full_row_blocks():
    """Wide shards: (col << rbits) does not fit 32 bits at 1024-row blocks, so the wide packs hold keys relative
    to one base per physical round (``wbase``) instead of shrinking the blocks to 2^(32 - bits(D)) rows. The
    logical entries decode to the same (column, row) pairs and the emulated product matches scipy; with bases
    off the builder falls back to the smaller blocks."""
    import numpy as np
    import scipy.sparse as sp
    import torch
    from photon_ml_amd.ops import tiled
    from photon_ml_amd.ops.tiled import TLFwdChunk
    rng = np.random.default_rng(0)
    n, d, k = 3000, 1 << 25, 30
    cols = np.concatenate([np.sort(rng.choice(d, k, replace=False)) for _ in range(n)])
    cols[::5] = rng.integers(0, 40, size=cols[::5].size)          # hot columns -> narrow rounds too
    x = sp.csr_matrix((rng.random(n * k) + 0.5, cols, np.arange(0, n * k + 1, k)), shape=(n, d))
    x.sum_duplicates()
    x.sort_indices()
    rp, c = torch.from_numpy(x.indptr.astype(np.int64)), torch.from_numpy(x.indices.astype(np.int64))
    v = torch.from_numpy(x.data)
    w = torch.from_numpy(rng.normal(size=d))
    ref = torch.from_numpy(x @ w.numpy())
    old = tiled.WIDE_BASE
    try:
        for wb in (0, 1):
            tiled.WIDE_BASE = wb
            ch = TLFwdChunk(rp, c, v, d)
            assert ch.rbits == (tiled.default_rbits(d, True) if wb else 32 - 25)
            assert (ch.wbase is not None) == bool(wb)
            torch.testing.assert_close(ch.emulate_matvec(w), ref, rtol=1e-12, atol=1e-12)
            pk, _ = ch.logical()
            assert int(pk.min()) >= 0 and int((pk >> ch.rbits).max()) < d
            if wb:
                # every stored relative key fits its 32 - rbits bits and every base is a column of its round
                rel = (ch.pack.to(torch.int64) & 0xFFFFFFFF) >> ch.rbits
                assert int(rel.max()) < 1 << (32 - ch.rbits) and int(ch.wbase.max()) < d
    finally:
        tiled.WIDE_BASE = old
