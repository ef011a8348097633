"""GAME on the GPU: fixed-effect coordinates on the HIP segmented-stream kernels and random-effect buckets solved
by the batched device solvers must reproduce the CPU (fp64 torch reference) results.

Reference behaviour: photon-api integTest ``GameEstimatorIntegTest`` (a full fit gives the same model whatever
the execution layout); numerics compared to the CPU path of this framework.
"""
import numpy as np
import pytest
import torch

from photon_ml_amd.data.game_data import generate_game_data
from photon_ml_amd.data.random_effect import FixedEffectDataConfiguration, RandomEffectDataConfiguration
from photon_ml_amd.estimators.game_estimator import GameEstimator
from photon_ml_amd.optimization.config import GLMOptimizationConfiguration, OptimizerConfig, RegularizationContext

pytestmark = pytest.mark.gpu


def _fit(device, task, data, opt="LBFGS", precision="f64"):
    cfg = GLMOptimizationConfiguration(OptimizerConfig(opt, 100, 1e-10), RegularizationContext("L2"), 1.0)
    est = (GameEstimator(device=device, precision=precision).set_training_task(task)
           .set_coordinate_data_configurations({"global": FixedEffectDataConfiguration("global"),
                                                "per-user": RandomEffectDataConfiguration("userId", "user"),
                                                "per-item": RandomEffectDataConfiguration("itemId", "item")})
           .set_coordinate_update_sequence(["global", "per-user", "per-item"])
           .set_coordinate_descent_iterations(2))
    return est.fit(data, data, [{"global": cfg, "per-user": cfg, "per-item": cfg}])[0]


@pytest.mark.parametrize("task", ["LOGISTIC_REGRESSION", "LINEAR_REGRESSION", "POISSON_REGRESSION"])
def test_game_fit_gpu_matches_cpu(task):
    assert torch.cuda.is_available()
    data, _ = generate_game_data(n_rows=4000, n_users=40, n_items=25, seed=21, task=task)
    rc = _fit("cpu", task, data)
    rg = _fit("cuda", task, data)
    wc = rc.model.get("global").glm.coefficients.means.cpu()
    wg = rg.model.get("global").glm.coefficients.means.cpu()
    assert torch.allclose(wc, wg, rtol=1e-5, atol=1e-6), (wc - wg).abs().max()
    for cid in ["per-user", "per-item"]:
        mc, mg = rc.model.get(cid), rg.model.get(cid)
        assert np.array_equal(mc.keys, mg.keys)
        np.testing.assert_allclose(mc.values, mg.values, rtol=1e-5, atol=1e-6)
    assert abs(rc.evaluations[0][1] - rg.evaluations[0][1]) < 1e-6


def test_game_fit_gpu_bf16_features_close():
    data, _ = generate_game_data(n_rows=4000, seed=22, task="LOGISTIC_REGRESSION")
    r64 = _fit("cuda", "LOGISTIC_REGRESSION", data)
    r16 = _fit("cuda", "LOGISTIC_REGRESSION", data, precision="bf16")
    assert abs(r64.evaluations[0][1] - r16.evaluations[0][1]) < 5e-3


@pytest.mark.parametrize("opt", ["TRON", "LBFGS"])
def test_segmented_random_effect_on_gpu_matches_cpu_dense(opt):
    """The block-diagonal random-effect solve on the HIP kernels == the dense CPU batch solve."""
    from photon_ml_amd.algorithm.coordinates import RandomEffectCoordinate
    data, _ = generate_game_data(n_rows=5000, n_users=60, seed=23, task="LOGISTIC_REGRESSION")
    cfg = GLMOptimizationConfiguration(OptimizerConfig(opt, 100, 1e-10), RegularizationContext("L2"), 1.0)
    cpu = RandomEffectCoordinate("u", data, RandomEffectDataConfiguration("userId", "user"), cfg,
                                 "LOGISTIC_REGRESSION", device="cpu", layout="dense")
    gpu = RandomEffectCoordinate("u", data, RandomEffectDataConfiguration("userId", "user"), cfg,
                                 "LOGISTIC_REGRESSION", device="cuda", layout="segmented")
    a, b = cpu.update_model(cpu.initialize_model()), gpu.update_model(gpu.initialize_model())
    for e in a.entity_ids[:20]:
        np.testing.assert_allclose(a.coefficients_of(e).means.numpy(), b.coefficients_of(e).means.numpy(),
                                   rtol=1e-5, atol=1e-6)
    sa, sb = cpu.score(a).cpu(), gpu.score(b).cpu()
    assert torch.allclose(sa, sb, atol=1e-5)


def test_game_model_scoring_on_device_matches_host():
    """FE / RE scoring on the device (cached CSR upload + segmented row reduction) == host scipy / torch, and
    repeated scoring of the same dataset reuses the device copy."""
    data, _ = generate_game_data(n_rows=3000, n_users=30, n_items=20, seed=24, task="LOGISTIC_REGRESSION")
    res = _fit("cpu", "LOGISTIC_REGRESSION", data, opt="TRON")
    model = res.model
    host = model.score(data, "cpu")
    dev1 = model.score(data, "cuda")
    dev2 = model.score(data, "cuda")
    assert dev1.is_cuda
    torch.testing.assert_close(dev1.cpu(), host, rtol=1e-12, atol=1e-12)
    assert torch.equal(dev1, dev2)
    x = data.shard(model.get("global").feature_shard_id)
    assert "cuda:0" in x._pml_dev_cache or "cuda" in x._pml_dev_cache


def test_scoring_kernel_paths_and_masks():
    """K5 / K6 HIP scoring kernel (score_rows_kernel): fixed and random effect, with a passive-row mask and
    entities without a model, == host scoring to fp64 rounding; deterministic."""
    from photon_ml_amd.ops.native import game_lib
    assert game_lib() is not None
    data, _ = generate_game_data(n_rows=4000, n_users=50, n_items=30, seed=25, task="LINEAR_REGRESSION")
    res = _fit("cpu", "LINEAR_REGRESSION", data, opt="TRON")
    rng = np.random.default_rng(0)
    mask = rng.random(data.n_rows) < 0.7
    for cid in ("global", "per-user", "per-item"):
        m = res.model.get(cid)
        kw = {} if cid == "global" else {"mask": mask}
        h = m.score(data, "cpu", **kw)
        d = m.score(data, "cuda", **kw)
        torch.testing.assert_close(d.cpu(), h, rtol=1e-12, atol=1e-12)
        assert torch.equal(d, m.score(data, "cuda", **kw))
    # rows whose entity has no model score 0
    sub = data.subset(np.arange(1000))
    re = res.model.get("per-user")
    from photon_ml_amd.models.game import RandomEffectModel
    keep = re.entity_ids[::2]
    idx = re.entity_index(keep)
    k, v = re.keys, re.values
    sel = np.isin(k // re.dim, idx)
    remap = {int(e): i for i, e in enumerate(idx)}
    nk = np.array([remap[int(a // re.dim)] * re.dim + int(a % re.dim) for a in k[sel]], dtype=np.int64)
    half = RandomEffectModel(re.random_effect_type, re.feature_shard_id, re.task, keep, re.dim, nk, v[sel])
    torch.testing.assert_close(half.score(sub, "cuda").cpu(), half.score(sub, "cpu"), rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (5, 40, 3), (100, 33, 64), (257, 129, 1000), (64, 2000, 17)])
def test_gemm_nt_mfma_matches_fp64(M, N, K):
    from photon_ml_amd.ops.native import gemm_nt
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g, device="cuda", dtype=torch.float64)
    B = torch.randn(N, K, generator=g, device="cuda", dtype=torch.float64)
    torch.testing.assert_close(gemm_nt(A, B), A @ B.T, rtol=1e-12, atol=1e-11 * max(1, K))


def test_random_projection_coordinate_on_gpu_matches_cpu():
    """RANDOM projector on the device: forward map X P^T (spmm_rows_kernel) and back-projection W P / V P^2
    (gemm_nt_mfma_kernel) give the CPU coordinate's coefficients, variances and scores."""
    from photon_ml_amd.algorithm.coordinates import RandomEffectCoordinate
    from photon_ml_amd.projector import RandomProjection
    data, _ = generate_game_data(n_rows=2000, n_users=12, d_user=30, seed=26, task="LINEAR_REGRESSION")
    cfg = GLMOptimizationConfiguration(OptimizerConfig("TRON", 50, 1e-10), RegularizationContext("L2"), 1.0)
    dc = RandomEffectDataConfiguration("userId", "user", projector_type=RandomProjection(6))
    out = {}
    for dev in ("cpu", "cuda"):
        c = RandomEffectCoordinate("u", data, dc, cfg, "LINEAR_REGRESSION", compute_variance=True, device=dev)
        m = c.update_model(c.initialize_model())
        out[dev] = (m, c.score(m).cpu())
    (a, sa), (b, sb) = out["cpu"], out["cuda"]
    for e in a.entity_ids:
        np.testing.assert_allclose(b.coefficients_of(e).means.numpy(), a.coefficients_of(e).means.numpy(),
                                   rtol=1e-7, atol=1e-9)
        np.testing.assert_allclose(b.coefficients_of(e).variances.numpy(), a.coefficients_of(e).variances.numpy(),
                                   rtol=1e-7, atol=1e-9)
    torch.testing.assert_close(sb, sa, rtol=1e-7, atol=1e-8)


@pytest.mark.parametrize("task", ["LOGISTIC_REGRESSION", "POISSON_REGRESSION"])
@pytest.mark.parametrize("d_user,proj", [(30, 6), (30, None), (90, None)])
def test_dense_buckets_fused_tron_match_batched_tron(task, d_user, proj, monkeypatch):
    """Dense size buckets (RANDOM projection, or INDEX_MAP on the dense layout) solved by the fused per-entity
    kernels (``entity_tron.DenseEntityTronBatch``: exact Hessian on the matrix cores for d <= 64, sparse
    Hessian-vector kernel above) == the batched-GEMM TRON (``batched.batched_tron``), across a warm start."""
    from photon_ml_amd.algorithm.coordinates import RandomEffectCoordinate
    from photon_ml_amd.projector import RandomProjection
    data, _ = generate_game_data(n_rows=6000, n_users=40, d_user=d_user, seed=27, task=task)
    # tolerance 1e-14: see test_fused_entity_tron_matches_pass_path
    cfg = GLMOptimizationConfiguration(OptimizerConfig("TRON", 100, 1e-14), RegularizationContext("L2"), 1.0)
    kw = {} if proj is None else {"projector_type": RandomProjection(proj)}
    dc = RandomEffectDataConfiguration("userId", "user", **kw)
    out = {}
    for fused in ("0", "1"):
        monkeypatch.setenv("PML_RE_FUSED", fused)
        c = RandomEffectCoordinate("u", data, dc, cfg, task, device="cuda", layout="dense")
        m1 = c.update_model(c.initialize_model())
        m2 = c.update_model(m1, partial_score=torch.from_numpy(np.cos(np.arange(data.n_rows)) * 0.2))
        assert bool(getattr(c, "_dense_fz", None)) == (fused == "1")
        out[fused] = (m1.values.copy(), m2.values.copy(), c.score(m2).cpu())
    for a, b in zip(out["0"], out["1"]):   # tolerances: see test_fused_entity_tron_matches_pass_path
        torch.testing.assert_close(torch.as_tensor(b), torch.as_tensor(a), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("cap,passive,ratio", [(20, 5, None), (7, 0, 0.05), (3, 2, 0.5)])
def test_random_effect_build_on_gpu_matches_host(cap, passive, ratio, monkeypatch):
    """Reservoir (K21), passive set and Pearson selection (K13) on the GPU (radix sorts, segment sums) == host."""
    from photon_ml_amd.data.random_effect import RandomEffectDataset
    data, _ = generate_game_data(n_rows=6000, n_users=40, d_user=24, seed=45, task="LOGISTIC_REGRESSION")
    cfg = RandomEffectDataConfiguration("userId", "user", active_data_upper_bound=cap,
                                        passive_data_lower_bound=passive, features_to_samples_ratio=ratio)
    monkeypatch.setenv("PML_RE_DEVICE_BUILD", "0")
    a = RandomEffectDataset(data, cfg, "cuda", layout="dense")
    monkeypatch.setenv("PML_RE_DEVICE_BUILD", "1")
    b = RandomEffectDataset(data, cfg, "cuda", layout="dense")
    assert b.device_build and not a.device_build
    assert np.array_equal(a.active_rows, b.active_rows) and np.array_equal(a.passive_rows, b.passive_rows)
    np.testing.assert_array_equal(a.weight_mult, b.weight_mult)
    xa, xb = a.x_active.tocsr(), b.x_active.tocsr()
    xa.sort_indices()
    xb.sort_indices()
    assert np.array_equal(xa.indptr, xb.indptr) and np.array_equal(xa.indices, xb.indices)


def test_row_space_gram_kernel_matches_indicator_passes(monkeypatch):
    """seg_gram_kernel (K_e from the block-diagonal CSR, one wave per entity) == the Gram columns formed by
    indicator passes through the transpose and forward GLM kernels, per size class; the solve on either set of
    factors gives the same model."""
    monkeypatch.setattr("photon_ml_amd.algorithm.coordinates.EAGER_SETUP", False)   # keeps the raw CSR
    from photon_ml_amd.algorithm.coordinates import RandomEffectCoordinate
    from photon_ml_amd.optimization.row_space import RowSpaceBatch
    data, _ = generate_game_data(n_rows=6000, n_users=400, d_user=40, seed=24, task="LOGISTIC_REGRESSION")
    cfg = GLMOptimizationConfiguration(OptimizerConfig("TRON", 60, 1e-10), RegularizationContext("L2"), 1.0)
    c = RandomEffectCoordinate("u", data, RandomEffectDataConfiguration("userId", "user"), cfg,
                               "LOGISTIC_REGRESSION", device="cuda", layout="segmented")
    ds = c.dataset
    a = RowSpaceBatch(ds.seg, csr=ds._seg_csr)
    b = RowSpaceBatch(ds.seg)
    assert a.B == b.B > 0 and len(a.classes) > 1 and [k.n for k in a.classes] == [k.n for k in b.classes]
    assert torch.equal(a.ents, b.ents)
    for ka, kb in zip(a.classes, b.classes):
        torch.testing.assert_close(ka.L, kb.L, rtol=1e-10, atol=1e-12)
    o = torch.zeros_like(ds.seg.y)
    ds.seg.o = o
    from photon_ml_amd.function.losses import LOGISTIC
    ra = a.solve(LOGISTIC, 1.0, "TRON", None, 1e-10, 60)
    rb = b.solve(LOGISTIC, 1.0, "TRON", None, 1e-10, 60)
    torch.testing.assert_close(a.to_primal(ra.W), b.to_primal(rb.W), rtol=1e-6, atol=1e-8)


def test_seg_gram_rows_per_round_bitwise(monkeypatch):
    """seg_gram_kernel with 1, 2, 4 or 8 rows per scatter round (interleaved image slots, one walk of row j per
    round): the same fma sequence per K entry, so K is bitwise equal for every S."""
    monkeypatch.setattr("photon_ml_amd.algorithm.coordinates.EAGER_SETUP", False)   # keeps the raw CSR
    from photon_ml_amd.algorithm.coordinates import RandomEffectCoordinate
    from photon_ml_amd.ops.native import require_game_lib, seg_gram
    from photon_ml_amd.optimization.row_space import _canonical_csr
    data, _ = generate_game_data(n_rows=8000, n_users=300, d_user=60, seed=5, task="LOGISTIC_REGRESSION")
    cfg = GLMOptimizationConfiguration(OptimizerConfig("TRON", 10, 1e-8), RegularizationContext("L2"), 1.0)
    c = RandomEffectCoordinate("u", data, RandomEffectDataConfiguration("userId", "user"), cfg,
                               "LOGISTIC_REGRESSION", device="cuda", layout="segmented")
    seg = c.dataset.seg
    csr = _canonical_csr(c.dataset._seg_csr, torch.device("cuda"))
    assert csr is not None
    n_e = seg.row_ptr[1:] - seg.row_ptr[:-1]
    ents = torch.nonzero((n_e > 0) & (n_e <= 64)).squeeze(1)
    n = int(n_e[ents].max())
    lib = require_game_lib()
    outs = []
    import os
    try:
        for S in (1, 2, 4, 8):
            lib.pml_seg_gram_set_s(S)
            for stage in ("0", "1"):     # entries read from global memory / staged in LDS first
                os.environ["PML_SEG_GRAM_STAGE"] = stage
                outs.append(seg_gram(ents, n, seg.row_ptr, seg.col_ptr, *csr))
    finally:
        lib.pml_seg_gram_set_s(0)
        os.environ.pop("PML_SEG_GRAM_STAGE", None)
    for K in outs[1:]:
        assert torch.equal(K, outs[0])
    assert float(outs[0].abs().sum()) > 0


@pytest.mark.parametrize("n", [1, 5, 8, 33, 64, 130])
def test_batched_cholesky_kernel(n):
    """batched_chol_kernel == torch.linalg.cholesky (fp64, 1e-12) on SPD Gram matrices with padding slots
    (rows >= nv[b] become the identity); a non-positive pivot is reported in info like LAPACK."""
    from photon_ml_amd.ops.native import batched_cholesky
    g = torch.Generator().manual_seed(n)
    B = 300
    X = torch.randn(B, n, n + 7, generator=g, dtype=torch.float64)
    K = X @ X.transpose(1, 2)
    nv = torch.randint(1, n + 1, (B,), generator=g)
    nv[0] = n
    ar = torch.arange(n)
    pad = ar.unsqueeze(0) >= nv.unsqueeze(1)
    Kp = torch.where(pad.unsqueeze(1) | pad.unsqueeze(2), torch.zeros(()), K) + torch.diag_embed(pad.double())
    ref = torch.linalg.cholesky(Kp)
    Kd = K.cuda().contiguous()
    if n > 1:
        Kd[1, 1, 1] = -1.0                      # not positive definite at column 2 (nv[1] may exclude it)
    L, info = batched_cholesky(Kd, nv.cuda())
    L, info = L.cpu(), info.cpu()
    keep = torch.ones(B, dtype=torch.bool)
    if n > 1:
        keep[1] = False
        assert int(info[1]) == (2 if int(nv[1]) >= 2 else 0)
    assert int(info[keep].abs().sum()) == 0
    torch.testing.assert_close(L[keep], ref[keep], rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("row_space", ["0", "1"])
def test_entity_masked_passes_give_identical_solve(row_space, monkeypatch):
    """The block-diagonal TRON skipping the row blocks / column tiles of entities that stopped iterating
    (DeviceGLMData.set_entity_mask) reproduces the full-pass solve bit for bit: active entities see the same
    entries in the same order; skipped outputs are never read."""
    import photon_ml_amd.optimization.batched as bt
    from photon_ml_amd.algorithm.coordinates import RandomEffectCoordinate
    monkeypatch.setenv("PML_RE_ROW_SPACE", row_space)
    monkeypatch.setenv("PML_RE_FUSED", "0")       # the pass path (the fused primal TRON reads no masked passes)
    data, _ = generate_game_data(n_rows=30000, n_users=500, d_user=8, seed=25, task="LOGISTIC_REGRESSION")
    cfg = GLMOptimizationConfiguration(OptimizerConfig("TRON", 30, 1e-10), RegularizationContext("L2"), 1.0)
    out = {}
    for masked in (False, True):
        monkeypatch.setattr(bt, "MASKED_PASSES", masked)
        c = RandomEffectCoordinate("u", data, RandomEffectDataConfiguration("userId", "user"), cfg,
                                   "LOGISTIC_REGRESSION", device="cuda", layout="segmented")
        m1 = c.update_model(c.initialize_model())
        m2 = c.update_model(m1, partial_score=torch.from_numpy(np.sin(np.arange(data.n_rows)) * 0.2))
        out[masked] = (m2.values.copy(), c.last_stats["mean_iterations"], c.score(m2).cpu())
    assert np.array_equal(out[False][0], out[True][0])
    assert out[False][1] == out[True][1]
    assert torch.equal(out[False][2], out[True][2])


def _re_two_updates(data, task, opt="TRON", max_iter=30, tol=1e-10):
    from photon_ml_amd.algorithm.coordinates import RandomEffectCoordinate
    cfg = GLMOptimizationConfiguration(OptimizerConfig(opt, max_iter, tol), RegularizationContext("L2"), 1.0)
    c = RandomEffectCoordinate("u", data, RandomEffectDataConfiguration("userId", "user"), cfg, task,
                               device="cuda", layout="segmented")
    m1 = c.update_model(c.initialize_model())
    s1 = c.score(m1).cpu()
    m2 = c.update_model(m1, partial_score=torch.from_numpy(np.sin(np.arange(data.n_rows)) * 0.2))
    return c, m1.values.copy(), s1, m2.values.copy(), c.score(m2).cpu()


@pytest.mark.parametrize("task", ["LOGISTIC_REGRESSION", "LINEAR_REGRESSION", "POISSON_REGRESSION"])
@pytest.mark.parametrize("max_rows", [None, 200])
@pytest.mark.parametrize("d_user,hess", [(12, 64), (12, 0), (40, 64), (100, 64)])
def test_fused_entity_tron_matches_pass_path(task, max_rows, d_user, hess, monkeypatch):
    """The fused per-entity primal TRON (one workgroup per entity, the whole solve in one launch) reproduces the
    block-diagonal pass-path TRON: same models, scores and iteration counts, across a warm-started second update.
    ``hess`` = HESS_DMAX: entities of <= 64 coefficients run the exact-Hessian kernel (re_tron_hess_kernel, MFMA;
    d_e 13 -> tile 16, 41 -> 48), wider ones (d_e 101) and hess = 0 the sparse Hessian-vector kernel.
    ``max_rows``: larger entities stay on the pass path (mixed components). TRON stops most entities on "function
    values converged" / "objective is not improving", where the point reached depends on rounding along the path
    (the exact Hessian, the fused and the pass-path Hessian-vector products all round differently): an objective
    resolved to ~1e-16 relative pins the coefficients only to ~sqrt(2e-16 f / lambda_min), ~1e-6 here. Measured
    for Poisson (``profiles/re_solver_agreement_poisson_d40.log``): the three solvers' models differ by up to 2e-6
    at tolerance 1e-10 and 3e-8 at 1e-14, with identical iteration counts and stop reasons."""
    import photon_ml_amd.optimization.entity_tron as et
    # power-law users (zipf): entities from a few rows (row space) to thousands (fused / pass path)
    data, _ = generate_game_data(n_rows=30000, n_users=700, d_user=d_user, seed=26, task=task)
    out = {}
    monkeypatch.setattr(et, "HESS_DMAX", hess)
    for fused in ("0", "1"):
        monkeypatch.setenv("PML_RE_FUSED", fused)
        monkeypatch.setattr(et, "FUSED_MAX_ROWS", max_rows or et.FUSED_MAX_ROWS)
        c, v1, s1, v2, s2 = _re_two_updates(data, task, max_iter=100, tol=1e-14)
        if fused == "1":
            rs, fz, sub = c._comps
            assert fz is not None and fz.B > 0
            assert (sub is not None) == (max_rows is not None)
            assert any(h for _, _, h in fz.launches) == (hess > 0 and d_user < 64)
        out[fused] = (v1, s1, v2, s2, c.last_stats["mean_iterations"])
    a, b = out["0"], out["1"]
    for i in range(4):
        torch.testing.assert_close(torch.as_tensor(b[i]), torch.as_tensor(a[i]), rtol=1e-5, atol=1e-6)
    assert abs(a[4] - b[4]) < 0.05


def test_fused_entity_tron_deterministic_and_matches_cpu(monkeypatch):
    """Bitwise-reproducible fused solve (fixed-order DPP wave sums, per-wave LDS accumulators), and the same
    model as the dense CPU batch solver (photon-api SingleNodeOptimizationProblem semantics per entity)."""
    from photon_ml_amd.algorithm.coordinates import RandomEffectCoordinate
    monkeypatch.setenv("PML_RE_FUSED", "1")
    data, _ = generate_game_data(n_rows=8000, n_users=80, d_user=10, seed=27, task="LOGISTIC_REGRESSION")
    r1 = _re_two_updates(data, "LOGISTIC_REGRESSION")
    r2 = _re_two_updates(data, "LOGISTIC_REGRESSION")
    assert r1[0]._comps[1] is not None
    assert np.array_equal(r1[3], r2[3]) and torch.equal(r1[4], r2[4])
    cfg = GLMOptimizationConfiguration(OptimizerConfig("TRON", 30, 1e-10), RegularizationContext("L2"), 1.0)
    cpu = RandomEffectCoordinate("u", data, RandomEffectDataConfiguration("userId", "user"), cfg,
                                 "LOGISTIC_REGRESSION", device="cpu", layout="dense")
    m = cpu.update_model(cpu.initialize_model())
    g = r1[0].update_model(None)
    for e in m.entity_ids[:30]:
        np.testing.assert_allclose(g.coefficients_of(e).means.numpy(), m.coefficients_of(e).means.numpy(),
                                   rtol=1e-5, atol=1e-6)


def test_row_space_gram_wide_entity_falls_back_to_indicator_passes(monkeypatch):
    """An entity with few rows but more projected columns than seg_gram_kernel's LDS image (d_e > SEG_GRAM_DMAX)
    gets its Gram columns from indicator passes; the other entities of its size class still use the kernel, and
    the factors match the all-indicator build."""
    monkeypatch.setattr("photon_ml_amd.algorithm.coordinates.EAGER_SETUP", False)   # keeps the raw CSR
    import scipy.sparse as sp
    from photon_ml_amd.algorithm.coordinates import RandomEffectCoordinate
    from photon_ml_amd.data.game_data import GameData
    from photon_ml_amd.ops.native import SEG_GRAM_DMAX
    from photon_ml_amd.optimization.row_space import RowSpaceBatch
    rng = np.random.default_rng(31)
    D = 3 * SEG_GRAM_DMAX
    rows, cols, vals, ids = [], [], [], []
    r = 0
    for e in range(40):
        n = 6 if e else 8
        width = (SEG_GRAM_DMAX // 3 + 500) if e == 0 else 20   # entity 0: 8 x 7.3K distinct columns > dmax
        for _ in range(n):
            c = rng.choice(D - 1, size=width, replace=False)
            rows += [r] * (width + 1)
            cols += sorted(c.tolist()) + [D - 1]
            vals += rng.normal(size=width).tolist() + [1.0]
            ids.append(e)
            r += 1
    x = sp.csr_matrix((vals, (rows, cols)), shape=(r, D))
    y = (rng.random(r) < 0.5).astype(float)
    data = GameData(y, {"user": x}, {"userId": np.array(ids)})
    cfg = GLMOptimizationConfiguration(OptimizerConfig("TRON", 30, 1e-10), RegularizationContext("L2"), 1.0)
    c = RandomEffectCoordinate("u", data, RandomEffectDataConfiguration("userId", "user"), cfg,
                               "LOGISTIC_REGRESSION", device="cuda", layout="segmented")
    ds = c.dataset
    d_e = ds.seg.col_ptr[1:] - ds.seg.col_ptr[:-1]
    assert int(d_e.max()) > SEG_GRAM_DMAX
    a = RowSpaceBatch(ds.seg, csr=ds._seg_csr)
    b = RowSpaceBatch(ds.seg)
    assert a.B == b.B == 40 and torch.equal(a.ents, b.ents)
    for ka, kb in zip(a.classes, b.classes):
        torch.testing.assert_close(ka.L, kb.L, rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("task", ["LOGISTIC_REGRESSION", "POISSON_REGRESSION"])
def test_resident_cluster_tron_matches_streaming(task, monkeypatch):
    """The register-resident fused TRON (rows in VGPRs; entities longer than one workgroup's rows solved by a
    CLUSTER of workgroups meeting at agent-scope barriers) reproduces the streaming fused kernel: same models to
    rounding and the same iteration counts, across a warm-started second update. ``force`` sends every eligible
    entity to it (the power-law users span 1 .. several clusters of 384 rows)."""
    import photon_ml_amd.optimization.entity_tron as et
    data, _ = generate_game_data(n_rows=60000, n_users=300, d_user=40, seed=28, task=task)
    out = {}
    for mode in ("0", "force"):
        monkeypatch.setattr(et, "RESIDENT", mode)
        monkeypatch.setattr(et, "HESS_DMAX", 0)          # d_e 41: the sparse kernels, not the tall one
        c, v1, s1, v2, s2 = _re_two_updates(data, task, max_iter=50, tol=1e-12)
        fz = c._comps[1]
        if mode == "force":
            assert fz.res is not None and fz.res["clusters"] > 0 and fz.res["n"] == fz.B
            t0 = fz.res["t0"].cpu()
            assert int((t0[1:] - t0[:-1]).max()) >= 8        # clusters of >= 8 member workgroups
        else:
            assert fz.res is None
        out[mode] = (v1, s1, v2, s2, c.last_stats["mean_iterations"])
    a, b = out["0"], out["force"]
    # the two kernels sum in different orders (8 vs 4 wave accumulators, member partials): models agree to the
    # rounding-path limit discussed in test_fused_entity_tron_matches_pass_path
    for i in range(4):
        torch.testing.assert_close(torch.as_tensor(b[i]), torch.as_tensor(a[i]), rtol=1e-5, atol=1e-6)
    assert abs(a[4] - b[4]) < 0.05


@pytest.mark.parametrize("task", ["LOGISTIC_REGRESSION", "POISSON_REGRESSION"])
def test_row_space_big_classes_match_primal(task, monkeypatch):
    """Wide entities of 64 < n_e <= 192 rows (d_e > n_e) are solved in their row space by rs_tron_big_kernel (one
    wave per problem, packed L in LDS; K_e from seg_gram_kernel, 3 rows per lane): same models, scores and
    iteration counts as the primal fused solve (the row-space map is an isometry: TRON takes the same steps)."""
    import scipy.sparse as sp
    from photon_ml_amd.data.game_data import GameData
    rng = np.random.default_rng(41)
    D, rows, cols, vals, ids = 4000, [], [], [], []
    r = 0
    sizes = [70, 90, 128, 150, 190, 66, 100] * 6
    for e, n in enumerate(sizes):
        pool = rng.choice(D - 1, size=400, replace=False)
        for _ in range(n):
            c = np.sort(rng.choice(pool, size=30, replace=False))
            rows += [r] * 31
            cols += c.tolist() + [D - 1]
            vals += rng.normal(size=30).tolist() + [1.0]
            ids.append(e)
            r += 1
    x = sp.csr_matrix((vals, (rows, cols)), shape=(r, D))
    z = np.asarray(x.sum(axis=1)).ravel() * 0.05
    y = (rng.random(r) < 1 / (1 + np.exp(-z))).astype(float) if task == "LOGISTIC_REGRESSION" else \
        rng.poisson(np.exp(np.clip(z, -3, 2))).astype(float)
    data = GameData(y, {"user": x}, {"userId": np.array(ids)})
    import photon_ml_amd.optimization.row_space as rsm
    out = {}
    monkeypatch.setenv("PML_RS_NMAX", "192")
    monkeypatch.setattr(rsm, "RS_BIG_NNZ_RATIO", 0.0)     # every wide entity in row space (sparse rows here)
    for rs in ("0", "1"):
        monkeypatch.setenv("PML_RE_ROW_SPACE", rs)
        c, v1, s1, v2, s2 = _re_two_updates(data, task, max_iter=50, tol=1e-12)
        if rs == "1":
            rsb = c._comps[0]
            assert rsb is not None and rsb.B == len(sizes) and max(cl.n for cl in rsb.classes) > 128
        out[rs] = (v1, s1, v2, s2, c.last_stats["mean_iterations"])
    a, b = out["0"], out["1"]
    for i in range(4):
        torch.testing.assert_close(torch.as_tensor(b[i]), torch.as_tensor(a[i]), rtol=1e-5, atol=1e-6)
    assert abs(a[4] - b[4]) < 0.05


@pytest.mark.parametrize("task,d_user", [("LOGISTIC_REGRESSION", 40), ("POISSON_REGRESSION", 40),
                                         ("LOGISTIC_REGRESSION", 700), ("LINEAR_REGRESSION", 300)])
def test_lean_streaming_tron_matches_csr_kernel(task, d_user, monkeypatch):
    """re_tron_lean_kernel (CG step / residual in registers, gradient in global scratch, W updated in place; only
    the gathered vector and the wave accumulators in LDS) runs the same sums in the same order as
    re_tron_csr_kernel: the same models, scores and iteration counts to rounding, across a warm-started second
    update, for every LDS class it serves (J = 1, 2, 4 coefficients per thread)."""
    import photon_ml_amd.ops.native as nat
    import photon_ml_amd.optimization.entity_tron as et
    data, _ = generate_game_data(n_rows=40000, n_users=200, d_user=d_user, seed=31, task=task)
    out = {}
    for lean in (0, 1024):
        monkeypatch.setattr(nat, "RE_LEAN_DMAX", lean)
        monkeypatch.setattr(et, "HESS_DMAX", 0)          # the sparse kernels, not the tall one
        monkeypatch.setenv("PML_RE_ROW_SPACE", "0")
        c, v1, s1, v2, s2 = _re_two_updates(data, task, max_iter=50, tol=1e-12)
        out[lean] = (v1, s1, v2, s2, c.last_stats["mean_iterations"])
    a, b = out[0], out[1024]
    for i in range(4):
        ta, tb = torch.as_tensor(a[i]), torch.as_tensor(b[i])
        print(f"max |diff| {float((ta - tb).abs().max()):.3e}")
        # fp-contraction may fuse differently around the register / global-memory vectors: rounding-level
        # differences, amplified along the TRON path as in test_fused_entity_tron_matches_pass_path
        torch.testing.assert_close(tb, ta, rtol=1e-5, atol=1e-6)
    assert abs(a[4] - b[4]) < 0.05


def test_row_space_classes_over_two_streams_match_one_stream(monkeypatch):
    """The opt-in multi-stream class path of the row-space solve (PML_RS_STREAMS > 1: classes dealt to side streams,
    warm starts / offsets recorded on them, None inputs skipped) gives bitwise the single-stream models and scores,
    over two updates (a cold and a warm start)."""
    import scipy.sparse as sp
    import photon_ml_amd.optimization.row_space as rsm
    from photon_ml_amd.data.game_data import GameData
    rng = np.random.default_rng(43)
    D, rows, cols, vals, ids = 3000, [], [], [], []
    r = 0
    sizes = [3, 7, 12, 16, 24, 30, 45, 60] * 8            # several size classes
    for e, n in enumerate(sizes):
        pool = rng.choice(D - 1, size=300, replace=False)
        for _ in range(n):
            c = np.sort(rng.choice(pool, size=20, replace=False))
            rows += [r] * 21
            cols += c.tolist() + [D - 1]
            vals += rng.normal(size=20).tolist() + [1.0]
            ids.append(e)
            r += 1
    x = sp.csr_matrix((vals, (rows, cols)), shape=(r, D))
    z = np.asarray(x.sum(axis=1)).ravel() * 0.05
    y = (rng.random(r) < 1 / (1 + np.exp(-z))).astype(float)
    data = GameData(y, {"user": x}, {"userId": np.array(ids)})
    out = {}
    for k in (1, 2):
        monkeypatch.setattr(rsm, "RS_STREAMS", k)
        c, v1, s1, v2, s2 = _re_two_updates(data, "LOGISTIC_REGRESSION", max_iter=30, tol=1e-10)
        rsb = c._comps[0]
        assert rsb is not None and len(rsb.classes) > 1
        if k == 2:
            assert getattr(rsb, "_streams", None)        # the side streams were used
        out[k] = (v1, s1, v2, s2)
    for a, b in zip(out[1], out[2]):
        assert torch.equal(torch.as_tensor(a), torch.as_tensor(b))


def test_fused_random_effect_update_never_builds_the_pass_layout():
    """With the fused solvers (row-space + per-entity primal TRON) an update, its scores and the materialised model
    need no pass over the whole random-effect coordinate: the block-diagonal pass layout (LazyGLMData) stays unbuilt
    (it is 0.6 s of game5pl's coordinate build); a pass-path consumer (the Hessian diagonal) then builds it once."""
    import scipy.sparse as sp
    from photon_ml_amd.data.game_data import GameData
    from photon_ml_amd.data.random_effect import LazyGLMData
    from photon_ml_amd.function.losses import loss_for_task
    rng = np.random.default_rng(47)
    D, rows, cols, vals, ids = 3000, [], [], [], []
    r = 0
    for e, n in enumerate([5, 12, 30, 90, 200, 260] * 6):   # row-space and fused primal entities
        pool = rng.choice(D - 1, size=300, replace=False)
        for _ in range(n):
            c = np.sort(rng.choice(pool, size=20, replace=False))
            rows += [r] * 21
            cols += c.tolist() + [D - 1]
            vals += rng.normal(size=20).tolist() + [1.0]
            ids.append(e)
            r += 1
    x = sp.csr_matrix((vals, (rows, cols)), shape=(r, D))
    y = (rng.random(r) < 0.4).astype(float)
    data = GameData(y, {"user": x}, {"userId": np.array(ids)})
    c, v1, s1, v2, s2 = _re_two_updates(data, "LOGISTIC_REGRESSION", max_iter=20, tol=1e-8)
    rs, fused, sub = c._comps
    assert rs is not None and fused is not None and sub is None
    glm = c.dataset.seg.glm
    assert isinstance(glm, LazyGLMData) and not glm.built
    assert np.isfinite(v2).all() and torch.isfinite(s2).all()
    W = torch.as_tensor(v2, device="cuda")
    h = c.dataset.seg.hdiag(loss_for_task("LOGISTIC_REGRESSION"), W, 1.0)
    assert glm.built and torch.isfinite(h).all() and bool((h >= 1.0 - 1e-12).all())
