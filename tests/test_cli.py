"""CLI driver tests (GameTrainingDriverIntegTest / GameScoringDriverIntegTest analogues, on CPU).

Reference: ``photon-client/src/integTest/.../cli/game/training/GameTrainingDriverIntegTest.scala`` (fixed-effect,
random-effect and mixed runs; output layout best/ + models/<i>/ with model-spec; hyper-parameter tuning adds
models; output modes) and ``GameScoringDriverIntegTest.scala`` (scores written as ScoringResultAvro and equal to
in-memory scoring). Data: synthetic GAME data written as Avro by :mod:`photon_ml_amd.io.data_writer`.
"""
import os

import numpy as np
import pytest

from photon_ml_amd.cli import game_scoring, game_training
from photon_ml_amd.cli.params import (expand_game_configurations, parse_coordinate_configuration,
                                      parse_feature_shard_configuration)
from photon_ml_amd.data.game_data import generate_game_data
from photon_ml_amd.io.data_writer import write_game_avro
from photon_ml_amd.io.score_io import load_scores

SHARDS = ["--feature-shard-configurations", "name=global,feature.bags=features",
          "--feature-shard-configurations", "name=user,feature.bags=userFeatures,intercept=true"]
FIXED = "name=fixed,feature.shard=global,optimizer=LBFGS,max.iter=50,tolerance=1e-8,regularization=L2,reg.weights=10|0.1"
RANDOM = ("name=per-user,feature.shard=user,random.effect.type=userId,optimizer=TRON,max.iter=20,tolerance=1e-8,"
          "regularization=L2,reg.weights=1")


@pytest.fixture(scope="module")
def game_avro(tmp_path_factory):
    root = tmp_path_factory.mktemp("game")
    data, _ = generate_game_data(n_rows=1500, n_users=20, seed=3, task="LOGISTIC_REGRESSION")
    tr, va = data.subset(np.arange(1200)), data.subset(np.arange(1200, 1500))
    bags = {"global": "features", "user": "userFeatures"}
    write_game_avro(str(root / "train"), tr, bags, n_files=2)
    write_game_avro(str(root / "val"), va, bags)
    return root


def test_dsl_parsing_and_grid():
    cc = parse_coordinate_configuration(FIXED + ",down.sampling.rate=0.5")
    cc.update(parse_coordinate_configuration(RANDOM.replace("reg.weights=1", "reg.weights=1|3")))
    fixed = cc["fixed"]
    assert not fixed.is_random_effect and fixed.optimization_configuration.down_sampling_rate == 0.5
    lams = [c.regularization_weight for c in fixed.expand_optimization_configurations()]
    assert lams == [10.0, 0.1]
    grid = expand_game_configurations(cc)
    assert len(grid) == 4 and {tuple(sorted(g)) for g in grid} == {("fixed", "per-user")}
    fs = parse_feature_shard_configuration("name=s,feature.bags=a|b,intercept=false")
    assert fs["s"].feature_bags == ["a", "b"] and not fs["s"].has_intercept
    with pytest.raises(ValueError):
        parse_coordinate_configuration("name=x,feature.shard=s")


def test_training_then_scoring(game_avro, tmp_path):
    out = tmp_path / "train-out"
    args = ["--input-data-directories", str(game_avro / "train"),
            "--validation-data-directories", str(game_avro / "val"),
            "--root-output-directory", str(out), "--training-task", "LOGISTIC_REGRESSION", *SHARDS,
            "--coordinate-configurations", FIXED, "--coordinate-configurations", RANDOM,
            "--coordinate-update-sequence", "fixed,per-user", "--coordinate-descent-iterations", "2",
            "--evaluators", "AUC,LOGISTIC_LOSS", "--output-mode", "ALL", "--device", "cpu",
            "--data-summary-directory", str(tmp_path / "summary"), "--data-validation", "VALIDATE_FULL"]
    res = game_training.GameTrainingDriver(game_training.build_parser().parse_args(args)).run()
    assert len(res["explicit"]) == 2 and res["best"] is not None
    aucs = [r.evaluations[0][1] for r in res["explicit"]]
    assert max(aucs) > 0.75
    assert res["best"].evaluations[0][1] == max(aucs)
    for d in ["best", "models/0", "models/1"]:
        assert os.path.exists(out / d / "model-metadata.json")
        assert os.path.exists(out / d / "model-spec")
        assert os.path.exists(out / d / "fixed-effect" / "fixed" / "coefficients" / "part-00000.avro")
        assert os.path.exists(out / d / "random-effect" / "per-user" / "id-info")
    assert os.path.exists(out / "logs" / "log-message.txt")
    assert os.path.exists(tmp_path / "summary" / "global" / "part-00000.avro")

    sout = tmp_path / "score-out"
    sargs = ["--input-data-directories", str(game_avro / "val"), "--root-output-directory", str(sout), *SHARDS,
             "--model-input-directory", str(out / "best"), "--model-id", "m1", "--evaluators", "AUC",
             "--device", "cpu"]
    sres = game_scoring.GameScoringDriver(game_scoring.build_parser().parse_args(sargs)).run()
    recs = load_scores(str(sout / "scores"))
    assert len(recs) == 300 and all(r["modelId"] == "m1" for r in recs)
    # scores of the saved model (coefficients < 1e-4 dropped) vs the in-memory best model
    best_val_auc = res["best"].evaluations[0][1]
    assert abs(sres["evaluations"][0][1] - best_val_auc) < 5e-3
    pred = np.array([r["predictionScore"] for r in recs])
    assert np.allclose(pred, sres["scores"].numpy() + sres["data"].offsets)
    # --spill-scores-to-disk: chunked scoring into a memory-mapped file gives the same scores / evaluation
    spout = tmp_path / "score-spill"
    spres = game_scoring.GameScoringDriver(game_scoring.build_parser().parse_args(
        [*sargs[:3], str(spout), *sargs[4:], "--spill-scores-to-disk", "true", "--spill-chunk-rows", "64"])).run()
    assert np.array_equal(spres["scores"].numpy(), sres["scores"].numpy())
    assert spres["evaluations"][0][1] == sres["evaluations"][0][1]
    assert [r["predictionScore"] for r in load_scores(str(spout / "scores"))] == list(pred)
    assert not [f for f in os.listdir(spout) if f.startswith(".scores-spill")]


def test_output_dir_exists_fails(game_avro, tmp_path):
    out = tmp_path / "o"
    out.mkdir()
    args = ["--input-data-directories", str(game_avro / "train"), "--root-output-directory", str(out),
            "--training-task", "LOGISTIC_REGRESSION", *SHARDS, "--coordinate-configurations", FIXED,
            "--coordinate-update-sequence", "fixed", "--coordinate-descent-iterations", "1", "--device", "cpu"]
    with pytest.raises(FileExistsError):
        game_training.GameTrainingDriver(game_training.build_parser().parse_args(args)).run()
    args += ["--override-output-directory", "true", "--output-mode", "EXPLICIT"]
    res = game_training.GameTrainingDriver(game_training.build_parser().parse_args(args)).run()
    # no validation data -> no evaluations; best falls back to the last explicit model
    assert len(res["explicit"]) == 2 and os.path.exists(out / "models" / "1" / "model-spec")


def test_hyperparameter_tuning_adds_models(game_avro, tmp_path):
    out = tmp_path / "tuned"
    args = ["--input-data-directories", str(game_avro / "train"),
            "--validation-data-directories", str(game_avro / "val"),
            "--root-output-directory", str(out), "--training-task", "LOGISTIC_REGRESSION", *SHARDS,
            "--coordinate-configurations", FIXED.replace("10|0.1", "1"),
            "--coordinate-update-sequence", "fixed", "--coordinate-descent-iterations", "1",
            "--hyper-parameter-tuning", "RANDOM", "--hyper-parameter-tuning-iterations", "3",
            "--output-mode", "TUNED", "--device", "cpu"]
    res = game_training.GameTrainingDriver(game_training.build_parser().parse_args(args)).run()
    assert len(res["tuned"]) == 3
    lams = {r.config["fixed"].regularization_weight for r in res["tuned"]}
    assert len(lams) == 3 and all(1e-4 <= l <= 1e4 for l in lams)
    assert sorted(os.listdir(out / "models")) == ["0", "1", "2"]


def test_feature_tools_index_and_bags(game_avro, tmp_path):
    from photon_ml_amd.cli import feature_tools
    from photon_ml_amd.io.index_map import OffHeapIndexMap, index_map_from_feature_bags
    a = feature_tools.build_parser().parse_args(
        ["index", "--input-data-directories", str(game_avro / "train"), "--root-output-directory",
         str(tmp_path / "idx"), "--num-storage-partitions", "3", *SHARDS])
    maps = feature_tools.run_indexing(a)
    assert maps["global"].feature_dimension == 20 and maps["user"].feature_dimension == 6
    b = feature_tools.build_parser().parse_args(
        ["bags", "--input-data-directories", str(game_avro / "train"), "--root-output-directory",
         str(tmp_path / "bags"), "--feature-bags-keys", "features,userFeatures"])
    keys = feature_tools.run_bags(b)
    assert len(keys["features"]) == 19 and open(tmp_path / "bags" / "features").read().count("\t") == 19
    im = index_map_from_feature_bags(str(tmp_path / "bags"), ["features"], True)
    assert im.feature_dimension == 20
    # training against the off-heap maps and then the bags directory gives the same model
    res = {}
    for i, opt in enumerate([["--off-heap-index-map-directory", str(tmp_path / "idx"),
                              "--off-heap-index-map-partitions", "3"],
                ["--feature-bags-directory", str(tmp_path / "bags")]]):
        out = tmp_path / f"o{i}"
        args = ["--input-data-directories", str(game_avro / "train"), "--root-output-directory", str(out),
                "--training-task", "LOGISTIC_REGRESSION", *SHARDS, "--coordinate-configurations",
                FIXED.replace("10|0.1", "1"), "--coordinate-update-sequence", "fixed",
                "--coordinate-descent-iterations", "1", "--device", "cpu", *opt]
        r = game_training.GameTrainingDriver(game_training.build_parser().parse_args(args)).run()
        m, maps_used = r["explicit"][0].model, r["index_maps"]["global"]
        w = m.get("fixed").glm.coefficients.means.numpy()
        res[opt[0]] = {maps_used.get_feature_name(j): w[j] for j in range(len(w))}
    a_, b_ = res.values()
    assert set(a_) == set(b_) and all(abs(a_[k] - b_[k]) < 1e-6 for k in a_)


def test_libsvm_to_avro_roundtrip(tmp_path):
    """dev-scripts/libsvm_text_to_trainingexample_avro.py analogue: LibSVM heart -> Avro -> same matrix."""
    from photon_ml_amd.io.data_reader import AvroDataReader, read_libsvm
    from photon_ml_amd.tools.libsvm_to_avro import convert
    src = "/root/reference/photon-client/src/integTest/resources/DriverIntegTest/input/heart.txt"
    n = convert(src, str(tmp_path / "heart"), records_per_file=100, binarize=True)
    assert n == 250 and len(os.listdir(tmp_path / "heart")) == 3
    ld_avro, im = AvroDataReader().read_labeled(str(tmp_path / "heart"))
    ld_txt, _ = read_libsvm(src, 13, binarize_labels=True)
    assert np.array_equal(ld_avro.y, ld_txt.y)
    # column j of the LibSVM matrix is feature name str(j + 1)
    for j in range(13):
        col = im.get_index(f"{j + 1}\u0001")
        np.testing.assert_allclose(ld_avro.x[:, col].toarray(), ld_txt.x[:, j].toarray())


@pytest.mark.parametrize("ext", ["json", "yaml"])
def test_config_file_round_trip(game_avro, tmp_path, ext):
    """``--config-file`` / ``--write-config``: the written options parse back to the same namespace, command-line
    flags replace the file's values (repeatable flags as a whole), and a run driven by a config file trains."""
    from photon_ml_amd.cli.params import load_config_file, parse_args_with_config
    out = tmp_path / "cfg-out"
    args = ["--input-data-directories", str(game_avro / "train"),
            "--root-output-directory", str(out), "--training-task", "LOGISTIC_REGRESSION", *SHARDS,
            "--coordinate-configurations", FIXED, "--coordinate-update-sequence", "fixed",
            "--coordinate-descent-iterations", "1", "--device", "cpu", "--compute-variance", "true"]
    cfg_path = str(tmp_path / f"train.{ext}")
    parser = game_training.build_parser()
    direct = parser.parse_args(args)
    written = parse_args_with_config(parser, args + ["--write-config", cfg_path])
    cfg = load_config_file(cfg_path)
    assert cfg["training-task"] == "LOGISTIC_REGRESSION" and len(cfg["feature-shard-configurations"]) == 2
    assert cfg["compute-variance"] is True
    from_file = parse_args_with_config(game_training.build_parser(), ["--config-file", cfg_path])
    for ns in (written, from_file):
        d, f = vars(direct), vars(ns)
        assert {k: v for k, v in f.items() if k not in ("config_file", "write_config")} == \
               {k: v for k, v in d.items() if k not in ("config_file", "write_config")}
    over = parse_args_with_config(game_training.build_parser(),
                                  ["--config-file", cfg_path, "--coordinate-descent-iterations", "3",
                                   "--feature-shard-configurations", "name=global,feature.bags=features"])
    assert over.coordinate_descent_iterations == 3 and len(over.feature_shard_configurations) == 1
    assert over.training_task == "LOGISTIC_REGRESSION"
    res = game_training.GameTrainingDriver(from_file).run()
    assert res["best"] is not None and os.path.exists(out / "best" / "model-metadata.json")
    with pytest.raises(ValueError):
        from photon_ml_amd.cli.params import config_to_argv
        config_to_argv(game_training.build_parser(), {"no-such-flag": 1})


def test_training_from_saved_model(game_avro, tmp_path):
    """``--model-input-directory`` on the training driver: a run initialised from a previous run's best model
    starts at (and stays near) that model's training loss instead of the zero model's."""
    base = ["--input-data-directories", str(game_avro / "train"), "--training-task", "LOGISTIC_REGRESSION", *SHARDS,
            "--coordinate-configurations", FIXED.replace("reg.weights=10|0.1", "reg.weights=1"),
            "--coordinate-configurations", RANDOM, "--coordinate-update-sequence", "fixed,per-user",
            "--device", "cpu"]
    first = game_training.GameTrainingDriver(game_training.build_parser().parse_args(
        base + ["--root-output-directory", str(tmp_path / "a"), "--coordinate-descent-iterations", "2"])).run()
    est_cold = game_training.GameTrainingDriver(game_training.build_parser().parse_args(
        base + ["--root-output-directory", str(tmp_path / "b"), "--coordinate-descent-iterations", "1"]))
    cold = est_cold.run()
    warm = game_training.GameTrainingDriver(game_training.build_parser().parse_args(
        base + ["--root-output-directory", str(tmp_path / "c"), "--coordinate-descent-iterations", "1",
                "--model-input-directory", str(tmp_path / "a" / "best")])).run()
    fw = first["best"].model.get("fixed").glm.coefficients.means
    ww = warm["best"].model.get("fixed").glm.coefficients.means
    cw = cold["best"].model.get("fixed").glm.coefficients.means
    # warm start from the converged 2-sweep model moves it far less than a cold 1-sweep run differs from it
    assert float(np.abs(np.asarray(ww) - np.asarray(fw)).max()) < 0.5 * float(np.abs(np.asarray(cw) - np.asarray(fw)).max())
