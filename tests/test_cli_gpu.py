"""CLI drivers end to end on the GPU (GAME training + scoring, legacy GLM driver) vs the same runs on the CPU
reference backend: the device path (HIP kernels, device-resident random effects, device evaluators) must give
the same models and metrics as the fp64 CPU path."""
import os

import numpy as np
import pytest

from photon_ml_amd.cli import game_scoring, game_training
from photon_ml_amd.data.game_data import generate_game_data
from photon_ml_amd.io.data_writer import write_game_avro

pytestmark = pytest.mark.gpu

SHARDS = ["--feature-shard-configurations", "name=global,feature.bags=features",
          "--feature-shard-configurations", "name=user,feature.bags=userFeatures,intercept=true"]
FIXED = "name=fixed,feature.shard=global,optimizer=LBFGS,max.iter=80,tolerance=1e-10,regularization=L2,reg.weights=1"
RANDOM = ("name=per-user,feature.shard=user,random.effect.type=userId,optimizer=TRON,max.iter=40,tolerance=1e-10,"
          "regularization=L2,reg.weights=1")


@pytest.fixture(scope="module")
def game_avro(tmp_path_factory):
    root = tmp_path_factory.mktemp("game_gpu")
    data, _ = generate_game_data(n_rows=3000, n_users=200, d_user=12, seed=13, task="LOGISTIC_REGRESSION")
    tr, va = data.subset(np.arange(2400)), data.subset(np.arange(2400, 3000))
    bags = {"global": "features", "user": "userFeatures"}
    write_game_avro(str(root / "train"), tr, bags, n_files=2)
    write_game_avro(str(root / "val"), va, bags)
    return root


def _train(game_avro, out, device, precision="f64"):
    args = ["--input-data-directories", str(game_avro / "train"),
            "--validation-data-directories", str(game_avro / "val"),
            "--root-output-directory", str(out), "--training-task", "LOGISTIC_REGRESSION", *SHARDS,
            "--coordinate-configurations", FIXED, "--coordinate-configurations", RANDOM,
            "--coordinate-update-sequence", "fixed,per-user", "--coordinate-descent-iterations", "2",
            "--evaluators", "AUC,LOGISTIC_LOSS", "--output-mode", "BEST", "--device", device]
    if precision != "f64":
        args += ["--precision", precision]
    return game_training.GameTrainingDriver(game_training.build_parser().parse_args(args)).run()


def test_game_training_and_scoring_cli_on_gpu_match_cpu(game_avro, tmp_path):
    cpu = _train(game_avro, tmp_path / "cpu", "cpu")
    gpu = _train(game_avro, tmp_path / "gpu", "cuda")
    a_cpu, a_gpu = cpu["best"].evaluations[0][1], gpu["best"].evaluations[0][1]
    assert a_gpu > 0.7 and abs(a_gpu - a_cpu) < 1e-6
    assert abs(cpu["best"].evaluations[1][1] - gpu["best"].evaluations[1][1]) < 1e-6 * abs(
        cpu["best"].evaluations[1][1])
    fe_c = cpu["best"].model.get("fixed").glm.coefficients.means.cpu().numpy()
    fe_g = gpu["best"].model.get("fixed").glm.coefficients.means.cpu().numpy()
    np.testing.assert_allclose(fe_g, fe_c, rtol=1e-5, atol=1e-7)
    sout = tmp_path / "score-out"
    sargs = ["--input-data-directories", str(game_avro / "val"), "--root-output-directory", str(sout), *SHARDS,
             "--model-input-directory", str(tmp_path / "gpu" / "best"), "--model-id", "g", "--evaluators", "AUC",
             "--device", "cuda"]
    sres = game_scoring.GameScoringDriver(game_scoring.build_parser().parse_args(sargs)).run()
    assert abs(sres["evaluations"][0][1] - a_gpu) < 5e-3
    assert os.path.exists(sout / "scores")
    # no --device: the scoring driver uses the GPU by default, and matches the CPU scores to fp64 rounding
    from photon_ml_amd.io.score_io import load_scores
    outs = {}
    for dev in (None, "cpu"):
        o = tmp_path / f"score-{dev}"
        args = sargs[:-2] + ([] if dev is None else ["--device", dev])
        args[args.index("--root-output-directory") + 1] = str(o)
        drv = game_scoring.GameScoringDriver(game_scoring.build_parser().parse_args(args))
        drv.run()
        outs[dev] = np.array([r["predictionScore"] for r in load_scores(str(o / "scores"))])
        assert drv.scoring_device.type == ("cuda" if dev is None else "cpu")
    np.testing.assert_allclose(outs[None], outs["cpu"], rtol=1e-10, atol=1e-10)


@pytest.mark.parametrize("norm,rtol", [("NONE", 5e-4), ("STANDARDIZATION", 1e-5)])
def test_legacy_driver_on_gpu_matches_cpu(tmp_path, norm, rtol):
    """photon-ml legacy Driver (heart.avro fixture, lambda path, validation, normalization) on cuda == cpu.
    TRON. Unnormalized, heart's raw features (e.g. cholesterol ~250 next to binary flags) make the optimum very
    flat in some directions: both backends stop on Photon's f-tolerance at points that differ by ~5e-5 there
    with equal objective; standardized, the problem is well conditioned and they agree to 1e-5."""
    from photon_ml_amd.cli import driver as drv
    # the reference's heart fixtures (copied into tests/fixtures: the GPU box has no /root/reference)
    ref = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures")
    models = {}
    for dev in ("cpu", "cuda"):
        args = ["--training-data-directory", f"{ref}/heart.avro", "--validating-data-directory",
                f"{ref}/heart_validation.avro", "--output-directory", str(tmp_path / dev), "--task",
                "LOGISTIC_REGRESSION", "--num-iterations", "100", "--convergence-tolerance", "1e-10",
                "--regularization-weights", "0.1,10", "--normalization-type", norm, "--optimizer", "TRON",
                "--device", dev]
        drv.Driver(drv.build_parser().parse_args(args)).run()
        models[dev] = drv.read_text_model(str(tmp_path / dev / drv.LEARNED_MODELS_TEXT))
    for lam in models["cpu"]:
        c, g = models["cpu"][lam], models["cuda"][lam]
        assert set(c) == set(g)
        for k in c:
            assert abs(c[k] - g[k]) <= rtol * max(1.0, abs(c[k])), (lam, k, c[k], g[k])


def test_game_training_from_saved_model_on_gpu(game_avro, tmp_path):
    """``--model-input-directory`` on the training driver with the device path: a saved (host) model initialises
    the cuda coordinates, and one more sweep from it matches the same warm start on the CPU backend."""
    first = _train(game_avro, tmp_path / "first", "cpu")
    assert first["best"] is not None
    outs = {}
    for dev in ("cpu", "cuda"):
        args = ["--input-data-directories", str(game_avro / "train"),
                "--validation-data-directories", str(game_avro / "val"),
                "--root-output-directory", str(tmp_path / f"warm-{dev}"), "--training-task", "LOGISTIC_REGRESSION",
                *SHARDS, "--coordinate-configurations", FIXED, "--coordinate-configurations", RANDOM,
                "--coordinate-update-sequence", "fixed,per-user", "--coordinate-descent-iterations", "1",
                "--evaluators", "AUC", "--device", dev, "--model-input-directory", str(tmp_path / "first" / "best")]
        outs[dev] = game_training.GameTrainingDriver(game_training.build_parser().parse_args(args)).run()
    a_c, a_g = outs["cpu"]["best"].evaluations[0][1], outs["cuda"]["best"].evaluations[0][1]
    assert a_g > 0.7 and abs(a_g - a_c) < 1e-6
