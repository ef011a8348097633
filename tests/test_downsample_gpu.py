"""Row-sampled shards (K20 down-sampling work saving, ``DeviceGLMData.row_sampled`` / ``tl_compact_kernel``).

The copy must hold exactly the kept rows' entries of every unit in the unit's logical order (bitwise), be
deterministic, pass the kernel-input validation, and give the same passes as the full shard with the dropped rows
at zero weight.
"""
import numpy as np
import pytest
import torch

from photon_ml_amd.function.losses import LOGISTIC

pytestmark = pytest.mark.gpu


def _filtered_logical(ch, keep: torch.Tensor, forward: bool, filt: bool):
    """The full chunk's logical entries (per unit: narrow, then wide) with the dropped rows' WIDE entries removed,
    and their narrow entries too when ``filt`` (else narrow sections are shared unfiltered)."""
    pk, vl = ch.logical()
    p = pk.to(torch.int64) & 0xFFFFFFFF
    t = ch._table().to(torch.int64).to(p.device)
    counts = ch.unit_counts().to(p.device)
    unit = torch.repeat_interleave(torch.arange(t.shape[0], device=p.device), counts)
    j = torch.arange(p.numel(), device=p.device) - (torch.cumsum(counts, 0) - counts)[unit]
    narrow = j < 256 * (t[:, 5] - t[:, 4])[unit]
    if forward:
        row = (unit << ch.rbits) + (p & ((1 << ch.rbits) - 1))
    else:
        row = p >> ch.cbits
    m = keep[row].bool() if filt else (narrow | keep[row].bool())
    return p[m], vl[m]


@pytest.mark.parametrize("filt", [False, True])
@pytest.mark.parametrize("precision", ["f64", "bf16"])
def test_row_sampled_shard_streams_and_passes(precision, filt, monkeypatch):
    """``filt``: the narrow rounds are filtered too (few rows kept) or shared (most rows kept)."""
    from photon_ml_amd.data.synthetic import generate_device_shard
    from photon_ml_amd.ops import device
    monkeypatch.setattr(device, "NARROW_FILTER_BELOW", 1.0 if filt else 0.0)
    data, _ = generate_device_shard(200_000, 50_000, 30, "cuda", precision, seed=6, chunk_rows=1 << 16,
                                    layout="tiled")
    assert sum(c.n_narrow_rounds for c in data.csr) > 0 and sum(c.n_narrow_rounds for c in data.csc) > 0
    g = torch.Generator(device="cuda").manual_seed(3)
    keep = torch.rand(data.n_rows, generator=g, device="cuda") < 0.3
    keep[70_000:140_000] = False                         # whole dropped blocks / a dropped chunk
    view = data.row_sampled(keep)
    assert view is not None and view.validate()
    kept_nnz = 0
    for c in range(len(data.csr)):
        kc = keep[data.row_starts[c]: data.row_starts[c + 1]]
        for full, samp, fwd in ((data.csr[c], view.csr[c], True), (data.csc[c], view.csc[c], False)):
            p0, v0 = _filtered_logical(full, kc, fwd, filt)
            p1, v1 = samp.logical()
            assert samp.n_narrow_rounds == (0 if filt else full.n_narrow_rounds) and samp.nnz == p0.numel()
            assert torch.equal(p1.to(torch.int64) & 0xFFFFFFFF, p0) and torch.equal(v1, v0)
        kept_nnz += view.csr[c].nnz
    if filt:
        assert 0 < kept_nnz < 0.35 * sum(c.nnz for c in data.csr)
    else:
        wide = sum(c.nnz - 256 * c.n_narrow_rounds for c in data.csr)
        assert 0 < kept_nnz - sum(256 * c.n_narrow_rounds for c in data.csr) < 0.35 * wide
    # the copy's shard-wide launch tables are derived from the full shard's (no rebuild)
    assert view._multi is not None and view._multi_t is not None
    # deterministic copy
    again = data.row_sampled(keep)
    for a, b in zip(view.csr + view.csc, again.csr + again.csc):
        assert torch.equal(a.pack, b.pack) and torch.equal(a.val, b.val)
    # passes == the full shard with the dropped rows at zero weight (shared weight vector)
    data.wt.mul_(keep.to(data.wt.dtype))
    data.mark_weights_changed()
    data.track_hessian = view.track_hessian = True
    w = (torch.randn(50_000, generator=torch.Generator().manual_seed(1), dtype=torch.float64) * 0.05).float()
    w = w.double().cuda()
    v = torch.randn(50_000, generator=torch.Generator().manual_seed(2), dtype=torch.float64).float().double().cuda()
    f0, s0, g0 = data.value_grad_sums(LOGISTIC, w, 0.01)
    f1, s1, g1 = view.value_grad_sums(LOGISTIC, w, 0.01)
    h0, _ = data.hv_sums(LOGISTIC, w, 0.01, v, 0.0)
    h1, _ = view.hv_sums(LOGISTIC, w, 0.01, v, 0.0)
    tol = 1e-12 if precision == "f64" else 1e-6
    assert abs(f1 - f0) <= tol * abs(f0) and abs(s1 - s0) <= tol * max(1.0, abs(s0))
    for a, b in ((g1, g0), (h1, h0)):
        assert torch.allclose(a, b, rtol=tol, atol=tol * float(b.abs().max()))
    z0 = data.margins(w)
    z1 = view.margins(w)
    assert torch.allclose(z1[keep], z0[keep], rtol=1e-12, atol=1e-12)


def test_fixed_effect_update_on_row_sampled_shard_matches_zero_weight_passes(monkeypatch):
    """A down-sampled fixed-effect update on the compacted shard == the same update with full zero-weight
    passes (same seed), and the compacted path is the one that ran."""
    from photon_ml_amd.algorithm.coordinates import FixedEffectCoordinate
    from photon_ml_amd.data.game_data import generate_game_data
    from photon_ml_amd.data.random_effect import FixedEffectDataConfiguration
    from photon_ml_amd.ops.device import DeviceGLMData
    from photon_ml_amd.optimization.config import GLMOptimizationConfiguration, OptimizerConfig, RegularizationContext
    from photon_ml_amd.sampling.samplers import reset_seed_sequence
    data, _ = generate_game_data(n_rows=20000, seed=8, task="LOGISTIC_REGRESSION")
    cfg = GLMOptimizationConfiguration(OptimizerConfig("LBFGS", 30, 1e-10), RegularizationContext("L2"), 1.0,
                                       down_sampling_rate=0.2)
    calls = []
    orig = DeviceGLMData.row_sampled

    def spy(self, keep):
        out = orig(self, keep)
        calls.append(out is not None)
        return out

    monkeypatch.setattr(DeviceGLMData, "row_sampled", spy)
    out = {}
    for compact in ("1", "0"):
        monkeypatch.setenv("PML_DS_COMPACT", compact)
        reset_seed_sequence()
        c = FixedEffectCoordinate("g", data, FixedEffectDataConfiguration("global"), cfg, "LOGISTIC_REGRESSION",
                                  device="cuda")
        m = c.update_model(c.initialize_model())
        m = c.update_model(m)                        # second update: a fresh sample, warm start
        out[compact] = m.glm.coefficients.means
        assert torch.equal(c.glm_data.wt.cpu().double(), torch.from_numpy(c.base_weights))
    assert calls == [True, True]
    torch.testing.assert_close(out["1"], out["0"], rtol=1e-7, atol=1e-9)
