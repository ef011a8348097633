"""Down-samplers (K20): BinaryClassificationDownSampler / DefaultDownSampler semantics
(photon-lib/.../sampler/*DownSampler.scala) with the counter-based row hash shared by host and device."""
import numpy as np
import pytest
import torch

from photon_ml_amd.sampling.samplers import (BinaryClassificationDownSampler, DefaultDownSampler, JavaRandom,
                                             down_sampler_for_task, reset_seed_sequence, row_uniforms)


def test_binary_down_sampler_semantics():
    rng = np.random.default_rng(0)
    y = (rng.random(20000) < 0.3).astype(float)
    w = rng.random(20000) + 0.5
    s = BinaryClassificationDownSampler(0.25, seed=7)
    out = s.sample_weights(y, w)
    pos = y == 1
    assert np.array_equal(out[pos], w[pos])                       # every positive kept as is
    kept = (~pos) & (out > 0)
    np.testing.assert_allclose(out[kept], w[kept] / 0.25)          # kept negatives re-weighted
    assert abs(kept.sum() / (~pos).sum() - 0.25) < 0.02
    # deterministic, and a row's decision depends only on (seed, row id)
    assert np.array_equal(out, s.sample_weights(y, w))
    ids = np.arange(20000)[::-1].copy()
    again = s.sample_weights(y[::-1], w[::-1], row_ids=ids)
    assert np.array_equal(again[::-1], out)


def test_default_down_sampler_and_factory():
    y = np.zeros(10000)
    w = np.ones(10000)
    out = DefaultDownSampler(0.4, seed=3).sample_weights(y, w)
    assert set(np.unique(out)) <= {0.0, 1.0} and abs(out.mean() - 0.4) < 0.03
    assert isinstance(down_sampler_for_task("LOGISTIC_REGRESSION", 0.5), BinaryClassificationDownSampler)
    assert isinstance(down_sampler_for_task("POISSON_REGRESSION", 0.5), DefaultDownSampler)
    with pytest.raises(ValueError):
        DefaultDownSampler(1.0)
    u = row_uniforms(1, np.arange(100000))
    assert 0.0 <= u.min() and u.max() < 1.0 and abs(u.mean() - 0.5) < 0.01


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("binary", [True, False])
def test_device_down_sampling_matches_host(dtype, binary):
    rng = np.random.default_rng(1)
    n = 100_003
    y = (rng.random(n) < 0.4).astype(float)
    w = rng.random(n) + 0.5
    ids = rng.permutation(10 * n)[:n].astype(np.int64)
    s = (BinaryClassificationDownSampler if binary else DefaultDownSampler)(0.3, seed=11)
    host = s.sample_weights(y, w.astype(np.float32).astype(float) if dtype == torch.float32 else w, row_ids=ids)
    dev = s.sample_weights_device(torch.from_numpy(y).to("cuda", dtype), torch.from_numpy(w).to("cuda", dtype),
                                  torch.from_numpy(ids).cuda())
    if dtype == torch.float64:
        assert np.array_equal(dev.cpu().numpy(), host)
    else:
        np.testing.assert_allclose(dev.cpu().double().numpy(), host, rtol=1e-6)
        assert np.array_equal(dev.cpu().numpy() > 0, host > 0)


@pytest.mark.gpu
def test_fixed_effect_down_sampling_gpu_matches_cpu():
    """A down-sampled fixed-effect update on the GPU (in-place weight rewrite) == the CPU update."""
    from photon_ml_amd.algorithm.coordinates import FixedEffectCoordinate
    from photon_ml_amd.data.game_data import generate_game_data
    from photon_ml_amd.data.random_effect import FixedEffectDataConfiguration
    from photon_ml_amd.optimization.config import (GLMOptimizationConfiguration, OptimizerConfig,
                                                   RegularizationContext)
    data, _ = generate_game_data(n_rows=4000, seed=8, task="LOGISTIC_REGRESSION")
    cfg = GLMOptimizationConfiguration(OptimizerConfig("TRON", 50, 1e-10), RegularizationContext("L2"), 1.0,
                                       down_sampling_rate=0.3)
    out = {}
    for dev in ("cpu", "cuda"):
        reset_seed_sequence()          # both updates draw the first seed of the reference sequence
        c = FixedEffectCoordinate("g", data, FixedEffectDataConfiguration("global"), cfg, "LOGISTIC_REGRESSION",
                                  device=dev)
        m = c.update_model(c.initialize_model())
        out[dev] = m.glm.coefficients.means.cpu()
        if dev == "cuda":   # full weights restored for scoring after the update
            assert torch.equal(c.glm_data.wt.cpu().double(), torch.from_numpy(c.base_weights))
    torch.testing.assert_close(out["cuda"], out["cpu"], rtol=1e-6, atol=1e-8)


def test_java_random_seed_sequence():
    """java.util.Random's nextLong, bit for bit (values of the JDK: new Random(42).nextInt() / nextLong())."""
    assert JavaRandom(42)._next(32) == -1170105035
    assert JavaRandom(42).next_long() == -5025562857975149833
    assert JavaRandom(0).next_long() == -4962768465676381896


def test_fresh_sample_per_fixed_effect_update():
    """Every down-sampling call draws a NEW seed from one Random(MathConst.RANDOM_SEED) sequence
    (photon-lib/.../sampler/DownSampler.scala:38-46), so successive fixed-effect updates see different samples —
    the seeds being the reference's nextLong() sequence."""
    from photon_ml_amd.algorithm.coordinates import FixedEffectCoordinate
    from photon_ml_amd.constants import RANDOM_SEED
    from photon_ml_amd.data.game_data import generate_game_data
    from photon_ml_amd.data.random_effect import FixedEffectDataConfiguration
    from photon_ml_amd.optimization.config import GLMOptimizationConfiguration, OptimizerConfig, RegularizationContext
    data, _ = generate_game_data(n_rows=3000, seed=9, task="LOGISTIC_REGRESSION")
    cfg = GLMOptimizationConfiguration(OptimizerConfig("LBFGS", 5, 1e-10), RegularizationContext("L2"), 1.0,
                                       down_sampling_rate=0.3)
    reset_seed_sequence()
    c = FixedEffectCoordinate("g", data, FixedEffectDataConfiguration("global"), cfg, "LOGISTIC_REGRESSION",
                              device="cpu")
    ref = JavaRandom(RANDOM_SEED)
    seen = []
    orig = c.sampler.sample_weights

    def spy(*a, **k):
        w = orig(*a, **k)
        seen.append((c.sampler.seed, w.copy()))
        return w

    c.sampler.sample_weights = spy
    m = c.update_model(c.initialize_model())
    c.update_model(m)
    assert [s for s, _ in seen] == [ref.next_long(), ref.next_long()]
    assert not np.array_equal(seen[0][1], seen[1][1])
    # a fixed-seed sampler (tests) keeps its sample
    s = BinaryClassificationDownSampler(0.3, seed=5)
    y, w = np.zeros(100), np.ones(100)
    assert np.array_equal(s.sample_weights(y, w), s.sample_weights(y, w))
