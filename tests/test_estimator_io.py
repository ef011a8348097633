"""Estimator, normalization and IO tests.

* GameEstimatorIntegTest.testNormalization (photon-api/src/integTest/.../estimators/GameEstimatorIntegTest.scala
  :129-178): every normalization type, no regularization -> scikit-learn coefficients to 1e-8.
* ModelProcessingUtilsTest save/load round trip; Avro codec round trips incl. reference files.
"""
import json
from collections import OrderedDict
import os

import numpy as np
import pytest
import torch

from photon_ml_amd.data.game_data import GameData, generate_game_data
from photon_ml_amd.data.random_effect import FixedEffectDataConfiguration, RandomEffectDataConfiguration
from photon_ml_amd.estimators.game_estimator import GameEstimator, GameTransformer, train_generalized_linear_model
from photon_ml_amd.io import avro
from photon_ml_amd.io.index_map import DefaultIndexMap
from photon_ml_amd.io.model_io import load_game_model, save_game_model, load_model_task
from photon_ml_amd.normalization.context import NormalizationContext, NormalizationType
from photon_ml_amd.optimization.config import GLMOptimizationConfiguration, OptimizerConfig, RegularizationContext
from photon_ml_amd.stat.summary import BasicStatisticalSummary

from test_optimizers import trivial_data

REF = "/root/reference/photon-client/src/integTest/resources"


@pytest.mark.parametrize("ntype", list(NormalizationType))
def test_normalization_matches_sklearn(ntype):
    ld = trivial_data()
    summary = BasicStatisticalSummary.compute(ld.x)
    norm = NormalizationContext.build(ntype, summary, intercept_id=2)
    res = train_generalized_linear_model(ld, "LINEAR_REGRESSION", "LBFGS", RegularizationContext("NONE"), [0.0],
                                         norm, max_iterations=100, tolerance=1e-11, device="cpu")
    w = res[0][1].coefficients.means.numpy()
    np.testing.assert_allclose(w, [0.34945501725815586, 0.26339479490270173, 0.4366125400310442], atol=1e-8)


def test_standardized_summary_known_values():
    ld = trivial_data()
    s = BasicStatisticalSummary.compute(ld.x)
    assert s.count == 10
    assert abs(float(s.mean[2]) - 1.0) < 1e-12 and float(s.variance[2]) == 0.0
    assert float(s.max[1]) == 0.0 and float(s.min[1]) < -0.89
    assert int(s.num_nonzeros[1]) == 4


def test_lambda_path_descending_warm_start():
    ld = trivial_data()
    res = train_generalized_linear_model(ld, "LOGISTIC_REGRESSION", "TRON", RegularizationContext("L2"),
                                         [0.1, 10.0, 1.0], device="cpu")
    assert [r[0] for r in res] == [10.0, 1.0, 0.1]
    norms = [float(r[1].coefficients.means.norm()) for r in res]
    assert norms[0] < norms[1] < norms[2]


def test_l1_sparsity_monotone_in_lambda():
    """DriverTest: number of non-zero coefficients non-increasing in the L1 weight."""
    from photon_ml_amd.data.synthetic import generate_glm_data
    ld, _ = generate_glm_data("LOGISTIC_REGRESSION", 800, 30, density=0.3, seed=1)
    res = train_generalized_linear_model(ld, "LOGISTIC_REGRESSION", "LBFGS", RegularizationContext("L1"),
                                         [0.1, 1, 10, 100], max_iterations=200, tolerance=1e-9, device="cpu")
    nnz = [int((r[1].coefficients.means.abs() > 0).sum()) for r in res]
    assert all(a <= b for a, b in zip(nnz, nnz[1:])), nnz  # lambdas descending -> nnz ascending


def test_avro_reference_model_file_and_roundtrip(tmp_path):
    p = f"{REF}/GameIntegTest/fixedEffectOnlyGAMEModel/fixed-effect/globalShard/coefficients/part-00000.avro"
    schema, recs = avro.read_records(p)
    assert schema["name"] == "BayesianLinearModelAvro" and len(recs) == 1
    assert recs[0]["modelClass"].endswith("LinearRegressionModel")
    means = recs[0]["means"]
    assert means[0]["name"] == "(INTERCEPT)"
    # sorted by |value| descending, all above threshold
    vals = [abs(m["value"]) for m in means]
    assert vals == sorted(vals, reverse=True) and min(vals) > 1e-4
    for codec in ("null", "deflate", "snappy"):
        out = tmp_path / f"m-{codec}.avro"
        avro.write_records(str(out), schema, recs, codec=codec)
        assert avro.read_records(str(out))[1] == recs


def test_load_reference_fixed_effect_model():
    d = f"{REF}/GameIntegTest/fixedEffectOnlyGAMEModel"
    recs = avro.read_records(f"{d}/fixed-effect/globalShard/coefficients/part-00000.avro")[1]
    keys = [f"{m['name']}\u0001{m['term']}" for m in recs[0]["means"]]
    im = DefaultIndexMap.from_keys(sorted(keys))
    model = load_game_model(d, {"globalShard": im})
    assert load_model_task(d).value == "LINEAR_REGRESSION"
    glm = model.get("globalShard").glm
    assert glm.task.value == "LINEAR_REGRESSION"
    assert abs(float(glm.coefficients.means[im.get_index("(INTERCEPT)\u0001")]) - 3.5525033712866567) < 1e-12


def test_game_model_save_load_roundtrip(tmp_path):
    data, _ = generate_game_data(n_rows=600, n_users=15, seed=8, task="LOGISTIC_REGRESSION")
    cfg = GLMOptimizationConfiguration(OptimizerConfig("TRON", 20, 1e-7), RegularizationContext("L2"), 1.0)
    est = (GameEstimator(device="cpu").set_training_task("LOGISTIC_REGRESSION")
           .set_coordinate_data_configurations({"global": FixedEffectDataConfiguration("global"),
                                                "per-user": RandomEffectDataConfiguration("userId", "user")})
           .set_coordinate_update_sequence(["global", "per-user"]).set_compute_variance(True))
    res = est.fit(data, data, [{"global": cfg, "per-user": cfg}])
    model = res[0].model
    maps = {s: DefaultIndexMap.from_keys([f"f{j}\u0001t" for j in range(data.shards[s].shape[1])])
            for s in data.shards}
    save_game_model(model, str(tmp_path / "m"), maps, opt_configs=res[0].config)
    meta = json.load(open(tmp_path / "m" / "model-metadata.json"))
    assert meta["modelType"] == "LOGISTIC_REGRESSION"
    assert open(tmp_path / "m" / "random-effect" / "per-user" / "id-info").read().split() == ["userId", "user"]
    loaded = load_game_model(str(tmp_path / "m"), maps)
    s0, _ = GameTransformer(model).transform(data)
    s1, ev = GameTransformer(loaded, ["AUC", "LOGISTIC_LOSS"]).transform(data)
    # coefficients below 1e-4 are dropped on save -> tiny score differences only
    assert torch.allclose(s0, s1, atol=5e-3)
    assert ev[0][1] > 0.7
    fe = loaded.get("global").glm.coefficients
    assert fe.variances is not None and bool((fe.variances > 0).all())


def test_avro_data_reader_heart():
    from photon_ml_amd.io.data_reader import AvroDataReader, FeatureShardConfiguration
    data, maps = AvroDataReader().read(f"{REF}/DriverIntegTest/input/heart.avro",
                                       {"s": FeatureShardConfiguration(["features"], True)})
    assert data.n_rows == 250 and data.shards["s"].shape == (250, 14)
    assert maps["s"].intercept_index == 13
    assert set(np.unique(data.response)) == {0.0, 1.0}


def test_snappy_codec_compresses_and_round_trips():
    """The OCF snappy writer emits real back-references (not literal-only streams) and decodes exactly,
    including incompressible data, overlapping copies and runs across 64 KiB fragment boundaries."""
    import os as _os
    from photon_ml_amd.io import avro
    nat = avro.native()
    rng = np.random.default_rng(3)
    cases = [b"", b"a", b"abcd" * 3, b"x" * 100000 + b"abc" * 777, rng.bytes(70000),
             b"".join(b"feature_%d\x01term\x00" % (i % 500) for i in range(20000)),
             rng.bytes(1000) * 80, b"ab" * 40000 + rng.bytes(3)]
    for c in cases:
        assert nat.snappy_roundtrip(c)
    text = cases[5]
    assert len(nat.snappy_compress(text)) < len(text) // 4
    noise = cases[4]
    assert len(nat.snappy_compress(noise)) <= len(noise) + len(noise) // 1000 + 16


def test_parallel_columnar_decode_is_deterministic(tmp_path, monkeypatch):
    """Files decoded on several threads merge in file order: same rows, same feature ids (first appearance),
    same bags as a single-threaded decode."""
    from photon_ml_amd.io import avro
    from photon_ml_amd.io.data_writer import game_example_schema
    rng = np.random.default_rng(5)
    schema = game_example_schema(["features", "other"])
    written = []
    for part in range(5):
        recs = []
        for i in range(200 + 37 * part):
            cols = rng.choice(300, 7, replace=False)
            recs.append({"uid": f"{part}-{i}", "response": float(i % 2), "weight": 1.0, "offset": 0.0,
                         "features": [{"name": f"f{c}", "term": "t", "value": float(c)} for c in cols],
                         "other": [{"name": f"o{part}", "term": "", "value": 1.0}], "metadataMap": {}})
        avro.write_records(str(tmp_path / f"part-{part}.avro"), schema, recs, codec="snappy" if part % 2 else "deflate")
        written.extend(recs)
    # a last file without the "other" bag: its rows have no "other" entries
    recs = [{"uid": f"x-{i}", "response": 1.0, "weight": 2.0, "offset": 0.5,
             "features": [{"name": "fz", "term": "", "value": 3.0}], "metadataMap": {}} for i in range(11)]
    avro.write_records(str(tmp_path / "part-9.avro"), game_example_schema(["features"]), recs)
    written.extend(recs)
    files = sorted(str(p) for p in tmp_path.iterdir())
    outs = []
    for th in ("1", "4"):
        monkeypatch.setenv("PML_AVRO_THREADS", th)
        outs.append(avro.native().read_columnar(files, ["response"], "weight", "offset", "uid", "metadataMap",
                                                ["features", "other"], [], "\x01"))
    a, b = outs
    assert a["n"] == b["n"] == sum(200 + 37 * p for p in range(5)) + 11
    assert list(a["vocab"]) == list(b["vocab"]) and list(a["uid"]) == list(b["uid"])
    for bag in ("features", "other"):
        for x, y in zip(a["bags"][bag], b["bags"][bag]):
            np.testing.assert_array_equal(x, y)
    # against the records themselves (row order = file order, first-appearance vocabulary)
    vocab = list(a["vocab"])
    assert list(a["uid"]) == [r["uid"] for r in written]
    np.testing.assert_array_equal(a["weight"], [r["weight"] for r in written])
    for bag in ("features", "other"):
        rp, keys, vals = a["bags"][bag]
        for i, r in enumerate(written):
            got = [(vocab[k], v) for k, v in zip(keys[rp[i]:rp[i + 1]], vals[rp[i]:rp[i + 1]])]
            assert got == [(f"{e['name']}\x01{e['term']}", e["value"]) for e in r.get(bag, [])], (bag, i)


def test_bags_to_csr_matches_coo_reference():
    """Direct CSR placement of bag entries (+ intercept, unmapped keys dropped) == the COO construction."""
    import scipy.sparse as sp
    from photon_ml_amd.io.data_reader import _bags_to_csr
    rng = np.random.default_rng(6)
    n, dim = 50, 40
    parts = []
    for pool in (np.r_[0:15, 30:40], np.r_[15:30, 40:50]):        # disjoint bags; keys >= 30 are unmapped
        cnt = rng.integers(0, 6, n)
        rowptr = np.r_[0, np.cumsum(cnt)]
        keys = np.concatenate([rng.choice(pool, c, replace=False) for c in cnt]).astype(np.int32)
        parts.append((rowptr, keys, rng.random(len(keys))))
    vocab_to_col = np.where(np.arange(60) < 30, np.arange(60), -1)
    m = _bags_to_csr(n, parts, vocab_to_col, dim, 39, True)
    rows, cols, vals = [], [], []
    for rowptr, keys, v in parts:
        rows.append(np.repeat(np.arange(n), np.diff(rowptr)))
        cols.append(vocab_to_col[keys])
        vals.append(v)
    rows.append(np.arange(n)); cols.append(np.full(n, 39)); vals.append(np.ones(n))
    r, c, v = map(np.concatenate, (rows, cols, vals))
    ok = c >= 0
    ref = sp.csr_matrix((v[ok], (r[ok], c[ok])), shape=(n, dim))
    ref.sort_indices()
    assert (m != ref).nnz == 0 and m.has_sorted_indices


@pytest.mark.parametrize("intercept", [True, False])
def test_native_shard_assembly_matches_python(intercept):
    """assemble_shard (C++, row ranges in parallel) == the numpy assembly: keys mapped through the index map
    (unmapped ones dropped), bags concatenated, the intercept appended, rows column-sorted; duplicates reported
    (first row / column) or summed."""
    from photon_ml_amd.io import data_reader as dr
    rng = np.random.default_rng(5)
    n, vocab, dim = 3000, 500, 400
    parts = []
    for _ in range(2):
        lens = rng.integers(0, 12, n)
        rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        keys = np.concatenate([rng.choice(vocab, size=l, replace=False) for l in lens]).astype(np.int32)
        parts.append((rp, keys, rng.normal(size=len(keys))))
    v2c = rng.permutation(vocab).astype(np.int64)
    v2c[v2c >= dim - 1] = -1              # keys outside the index map are dropped (dim - 1: the intercept)
    # two bags may hold the same feature: make the columns of the second bag disjoint to test the clean path
    v2c_b = v2c.copy()
    icpt = dim - 1 if intercept else None
    clean = [parts[0], (parts[1][0], parts[1][1], parts[1][2])]
    ref = dr._bags_to_csr(n, [parts[0]], v2c_b, dim, icpt, True)
    got = dr._assemble(n, [parts[0]], v2c_b, dim, icpt, True)
    assert np.array_equal(ref.indptr, got.indptr) and np.array_equal(ref.indices, got.indices)
    assert np.array_equal(ref.data, got.data)
    with pytest.raises(dr.DuplicateFeatureError) as e1:
        dr._bags_to_csr(n, clean, v2c, dim, icpt, True)
    with pytest.raises(dr.DuplicateFeatureError) as e2:
        dr._assemble(n, clean, v2c, dim, icpt, True)
    assert str(e1.value) == str(e2.value)
    a = dr._bags_to_csr(n, clean, v2c, dim, icpt, False)
    b = dr._assemble(n, clean, v2c, dim, icpt, False)
    assert np.array_equal(a.indptr, b.indptr) and np.array_equal(a.indices, b.indices)
    np.testing.assert_allclose(a.data, b.data, rtol=1e-15, atol=0)


def test_native_model_writer_is_byte_identical(tmp_path, monkeypatch):
    """save_game_model with the native BayesianLinearModel encoder (io/model_io.write_linear_models) writes the
    same bytes as the per-record Python dictionaries: fixed effect with variances, random effect over several
    files, tiny coefficients dropped, |w| ordering with ties."""
    import filecmp
    from photon_ml_amd.constants import TaskType
    from photon_ml_amd.io import model_io
    from photon_ml_amd.io.index_map import DefaultIndexMap
    from photon_ml_amd.models.game import FixedEffectModel, GameModel, RandomEffectModel
    from photon_ml_amd.models.glm import Coefficients, model_for_task
    rng = np.random.default_rng(4)
    D = 300
    im = DefaultIndexMap.from_keys([f"f{j}\u0001t{j % 4}" for j in range(D)] + ["(INTERCEPT)\u0001"])
    task = TaskType.LOGISTIC_REGRESSION
    w = rng.normal(size=D + 1)
    w[::9] = 1e-7
    w[5] = w[6]
    fe = FixedEffectModel(model_for_task(task, Coefficients(torch.from_numpy(w), torch.from_numpy(rng.random(D + 1)))),
                          "g")
    n_ent = 23
    keys, vals = [], []
    for e in range(n_ent):
        f = np.sort(rng.choice(D + 1, size=int(rng.integers(0, 30)), replace=False))
        keys.append(e * (D + 1) + f)
        vals.append(rng.normal(size=f.size) * np.where(rng.random(f.size) < 0.2, 1e-6, 1.0))
    re = RandomEffectModel("userId", "g", task, np.array([f"u{e}" for e in range(n_ent)]), D + 1,
                           np.concatenate(keys), np.concatenate(vals))
    model = GameModel(OrderedDict([("fixed", fe), ("per-user", re)]))
    for flag, out in (("1", tmp_path / "native"), ("0", tmp_path / "python")):
        monkeypatch.setattr(model_io, "NATIVE_MODEL_WRITER", flag == "1")
        model_io.save_game_model(model, str(out), {"g": im}, task=task, entities_per_file=7)
    cmp = filecmp.dircmp(tmp_path / "native", tmp_path / "python")

    def same(c):
        assert not c.left_only and not c.right_only and not c.diff_files, (c.left, c.diff_files)
        (_, mismatch, errors) = filecmp.cmpfiles(c.left, c.right, c.common_files, shallow=False)
        assert not mismatch and not errors, mismatch
        for sub in c.subdirs.values():
            same(sub)
    same(cmp)


def test_sorted_factors_match_np_unique():
    """The random-effect build's entity ids from a factorisation (reader codes / pandas) equal np.unique of the
    per-row strings; values that print alike (1 and "1") fall back to the per-row path."""
    from photon_ml_amd.data.random_effect import factorize_ids, sorted_factors
    rng = np.random.default_rng(3)
    table = np.array(["u10", "u2", "b", "ä", "u1", "", "zz"], dtype=object)
    codes = rng.integers(0, len(table), 500)
    ids = table[codes]
    u, inv = sorted_factors(codes, table)
    ru, rinv = np.unique(ids.astype(str), return_inverse=True)
    assert np.array_equal(u, ru) and np.array_equal(inv, rinv)
    u, inv = factorize_ids(ids)
    assert np.array_equal(u, ru) and np.array_equal(inv, rinv)
    assert factorize_ids(np.array([1, "1", "x"], dtype=object)) is None          # 1 and "1" print alike
    assert factorize_ids(np.array(["a", None, "b"], dtype=object)) is None       # missing values


def test_reader_vocab_map_is_the_sorted_key_map():
    """The reader's sort-based vocabulary map equals DefaultIndexMap.from_keys(sorted(used keys)) + lookups."""
    from photon_ml_amd.constants import INTERCEPT_KEY
    from photon_ml_amd.io.data_reader import _sorted_vocab_map
    from photon_ml_amd.io.index_map import DefaultIndexMap
    rng = np.random.default_rng(5)
    vocab = [f"f{int(v)}\u0001t{int(v) % 3}" for v in rng.permutation(2000)] + ["é\u0001", "Z\u0001", "a b\u0001x"]
    used = np.sort(rng.choice(len(vocab), 700, replace=False))
    for icpt in (False, True):
        im, v2c = _sorted_vocab_map(vocab, used, icpt)
        ref = DefaultIndexMap.from_keys(sorted(vocab[i] for i in used), add_intercept=icpt)
        assert im.index_to_key == ref.index_to_key
        assert np.array_equal(v2c, ref.get_indices(vocab))
        assert im.get_index(INTERCEPT_KEY) == ref.get_index(INTERCEPT_KEY)
    # the intercept key present in the data: the dictionary path, same result
    vocab2 = vocab + [INTERCEPT_KEY]
    used2 = np.append(used, len(vocab2) - 1)
    im, v2c = _sorted_vocab_map(vocab2, used2, True)
    ref = DefaultIndexMap.from_keys(sorted(vocab2[i] for i in used2), add_intercept=True)
    assert im.index_to_key == ref.index_to_key and np.array_equal(v2c, ref.get_indices(vocab2))
