"""GAME training driver (command line).

Reference: ``photon-client/.../cli/game/GameDriver.scala:43-260`` (shared params, feature-map preparation from an
off-heap index map directory or a feature-bags directory, date-range input paths) and
``cli/game/training/GameTrainingDriver.scala:63-720``:

  clean output dirs -> feature maps -> read train / validation -> validate -> per-shard statistics (written to
  ``--data-summary-directory/<shard>``) -> normalization contexts -> λ grid (cartesian product over coordinates)
  -> ``GameEstimator.fit`` -> optional hyper-parameter tuning (needs validation data) -> select models by the first
  validation evaluator -> save ``best/`` and ``models/<i>/`` (each with a ``model-spec`` text file).

Usage::

    python -m photon_ml_amd.cli.game_training \\
        --input-data-directories train/ --validation-data-directories val/ --root-output-directory out/ \\
        --training-task LOGISTIC_REGRESSION \\
        --feature-shard-configurations name=global,feature.bags=features \\
        --feature-shard-configurations name=user,feature.bags=userFeatures,intercept=true \\
        --coordinate-configurations name=fixed,feature.shard=global,optimizer=LBFGS,max.iter=50,tolerance=1e-7,\\
regularization=L2,reg.weights=0.1|1|10 \\
        --coordinate-configurations name=per-user,feature.shard=user,random.effect.type=userId,optimizer=TRON,\\
max.iter=20,tolerance=1e-7,regularization=L2,reg.weights=1 \\
        --coordinate-update-sequence fixed,per-user --coordinate-descent-iterations 2 --evaluators AUC

Multi-GPU: launch with ``torchrun``; each rank reads its slice of the input files and the fixed-effect solves
all-reduce one packed buffer per evaluation over RCCL (see :mod:`photon_ml_amd.parallel.dist`). Index maps must then
come from ``--feature-bags-directory`` or ``--off-heap-index-map-directory`` so every rank agrees on them.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
from collections import OrderedDict
from typing import Dict, List, Optional

import numpy as np

from ..data.random_effect import RandomEffectDataConfiguration
from ..data.validators import DataValidationType, sanity_check
from ..estimators.game_estimator import GameEstimator, GameResult
from ..hyperparameter.game_tuning import GameEstimatorEvaluationFunction
from ..hyperparameter.search import DoubleRange, GaussianProcessSearch, RandomSearch
from ..io.avro import avro_files
from ..io.data_reader import AvroDataReader, InputColumnNames
from ..io.index_map import index_map_from_feature_bags, open_index_map
from ..io.model_io import save_game_model
from ..io.score_io import save_feature_summary
from ..normalization.context import NormalizationContext, NormalizationType
from ..parallel.dist import is_dist, rank, world_size
from ..stat.summary import BasicStatisticalSummary
from ..utils.logging_utils import PhotonLogger
from ..utils.timing import Timed
from .params import (HyperparameterTuningMode, ModelOutputMode, add_config_arguments, coordinate_configuration_to_string,
                     expand_daily_dirs, expand_game_configurations, parse_bool, parse_coordinate_configuration,
                     parse_args_with_config, parse_date_range, parse_days_range, parse_feature_shard_configuration, parse_kv,
                     split_list)

MODELS_DIR = "models"
MODEL_SPEC_DIR = "model-spec"
BEST_MODEL_DIR = "best"
LOGS = "logs"
DEFAULT_APPLICATION_NAME = "GAME-Training"


def add_common_arguments(p: argparse.ArgumentParser):
    """GameDriver.scala:55-125 parameters."""
    p.add_argument("--input-data-directories", action="append", required=True)
    p.add_argument("--input-data-date-range")
    p.add_argument("--input-data-days-range")
    p.add_argument("--off-heap-index-map-directory")
    p.add_argument("--off-heap-index-map-partitions", type=int)
    p.add_argument("--input-column-names")
    p.add_argument("--evaluators", "--validation-evaluators", dest="evaluators", action="append")
    p.add_argument("--root-output-directory", required=True)
    p.add_argument("--override-output-directory", type=parse_bool, default=False)
    p.add_argument("--output-files-limit", type=int)
    p.add_argument("--feature-bags-directory")
    p.add_argument("--feature-shard-configurations", action="append", required=True)
    p.add_argument("--data-validation", default="VALIDATE_DISABLED")
    p.add_argument("--logging-level", default="INFO")
    p.add_argument("--application-name", default=DEFAULT_APPLICATION_NAME)
    p.add_argument("--device", default=None, help="torch device (default: cuda if available)")
    p.add_argument("--precision", default="f64", choices=["bf16", "f32", "f64"],
                   help="fixed-effect feature storage precision on the GPU (accumulation is always fp64)")
    add_config_arguments(p)


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="game-training", description=__doc__.split("\n")[0])
    add_common_arguments(p)
    p.add_argument("--training-task", required=True)
    p.add_argument("--validation-data-directories", action="append")
    p.add_argument("--validation-data-date-range")
    p.add_argument("--validation-data-days-range")
    p.add_argument("--minimum-validation-partitions", type=int, default=1)
    p.add_argument("--output-mode", default="BEST")
    p.add_argument("--coordinate-configurations", action="append", required=True)
    p.add_argument("--coordinate-update-sequence", required=True)
    p.add_argument("--coordinate-descent-iterations", type=int, required=True)
    p.add_argument("--normalization", default="NONE")
    p.add_argument("--data-summary-directory")
    p.add_argument("--tree-aggregate-depth", type=int, default=1,
                   help="reduction depth of the reference's treeAggregate: >= 2 selects RCCL's tree all-reduce "
                        "(unless --allreduce-algo says otherwise), 1 leaves the choice to RCCL")
    p.add_argument("--allreduce-algo", choices=["auto", "ring", "tree"], default=None,
                   help="RCCL all-reduce algorithm of the gradient reduction (NCCL_ALGO); default: from "
                        "--tree-aggregate-depth")
    p.add_argument("--hyper-parameter-tuning", default="NONE")
    p.add_argument("--hyper-parameter-tuning-iterations", type=int, default=0)
    p.add_argument("--hyper-parameter-tuning-range", default="1e-4-1e4")
    p.add_argument("--hyper-parameter-tuning-scale", default="LOG", choices=["LOG", "LINEAR"])
    p.add_argument("--compute-variance", type=parse_bool, default=False)
    p.add_argument("--use-warm-start", type=parse_bool, default=True)
    p.add_argument("--checkpoint-directory", help="save coordinate-descent state after every coordinate update")
    p.add_argument("--model-input-directory",
                   help="initialise training from a saved GAME model directory (e.g. a previous run's best/)")
    p.add_argument("--resume", type=parse_bool, default=False,
                   help="continue an interrupted run from --checkpoint-directory (the output directory is kept)")
    return p


def process_output_dir(path: str, override: bool):
    """IOUtils.processOutputDir: fail if it exists unless overriding (then delete)."""
    if os.path.exists(path):
        if not override:
            raise FileExistsError(f"Output directory {path} already exists and override is not set")
        if rank() == 0:
            shutil.rmtree(path)
    if is_dist():
        from ..parallel.dist import barrier
        barrier()


def resolve_paths(dirs: List[str], date_range: Optional[str], days_range: Optional[str]) -> List[str]:
    """IOUtils.resolveRange + getInputPathsWithinDateRange (date and days ranges are mutually exclusive)."""
    dirs = split_list(dirs)
    if date_range and days_range:
        raise ValueError("Both date range and days range given; pick one")
    if date_range:
        return expand_daily_dirs(dirs, *parse_date_range(date_range))
    if days_range:
        return expand_daily_dirs(dirs, *parse_days_range(days_range))
    return dirs


def rank_files(paths: List[str]) -> List[str]:
    """This rank's slice of the input files (round-robin by sorted file name)."""
    files = avro_files(paths)
    if not is_dist():
        return files
    mine = files[rank()::world_size()]
    if not mine:
        raise ValueError(f"rank {rank()} has no input files ({len(files)} files for {world_size()} ranks)")
    return mine


class GameDriverBase:
    def __init__(self, args: argparse.Namespace):
        self.args = args
        self.shard_configs = OrderedDict()
        for s in args.feature_shard_configurations:
            self.shard_configs.update(parse_feature_shard_configuration(s))
        self.columns = InputColumnNames()
        if args.input_column_names:
            self.columns.update(parse_kv(args.input_column_names))
        if (args.off_heap_index_map_directory is None) != (args.off_heap_index_map_partitions is None):
            raise ValueError("Off-heap index map directory and partitions must be given together")
        if args.off_heap_index_map_directory and args.feature_bags_directory:
            raise ValueError("Ambiguous index map input: both off-heap index map directory and feature bags directory")
        self.logger: Optional[PhotonLogger] = None

    def log(self, msg, level="info"):
        if self.logger is not None:
            getattr(self.logger, level)(msg)

    def prepare_feature_maps(self):
        a = self.args
        if a.off_heap_index_map_directory:
            return {sid: open_index_map(a.off_heap_index_map_directory, sid, a.off_heap_index_map_partitions)
                    for sid in self.shard_configs}
        if a.feature_bags_directory:
            return {sid: index_map_from_feature_bags(a.feature_bags_directory, cfg.feature_bags, cfg.has_intercept)
                    for sid, cfg in self.shard_configs.items()}
        if is_dist():
            raise ValueError("multi-rank runs need --feature-bags-directory or --off-heap-index-map-directory")
        return None

    def id_tags(self) -> List[str]:
        return []

    def read(self, paths, index_maps):
        # training never reports per-record uids (scores are written by game-scoring): skip their strings
        return AvroDataReader(self.columns).read(rank_files(paths), self.shard_configs, index_maps, self.id_tags(),
                                                 uids=False)


class GameTrainingDriver(GameDriverBase):
    def __init__(self, args: argparse.Namespace):
        super().__init__(args)
        self.coord_configs = OrderedDict()
        for s in args.coordinate_configurations:
            self.coord_configs.update(parse_coordinate_configuration(s))
        self.update_sequence = split_list([args.coordinate_update_sequence])
        self.output_mode = ModelOutputMode(args.output_mode.upper())
        self.tuning = HyperparameterTuningMode(args.hyper_parameter_tuning.upper())
        self.normalization = NormalizationType.parse(args.normalization)
        self.validate_params()

    def validate_params(self):
        missing = [c for c in self.update_sequence if c not in self.coord_configs]
        if missing:
            raise ValueError(f"Coordinates {missing} in the update sequence have no configuration")
        for cid, cc in self.coord_configs.items():
            if cc.data_configuration.feature_shard_id not in self.shard_configs:
                raise ValueError(f"Coordinate {cid} uses undefined feature shard "
                                 f"{cc.data_configuration.feature_shard_id}")
        if self.tuning != HyperparameterTuningMode.NONE and self.args.hyper_parameter_tuning_iterations <= 0:
            raise ValueError("hyper-parameter tuning needs --hyper-parameter-tuning-iterations > 0")
        if self.args.coordinate_descent_iterations <= 0:
            raise ValueError("coordinate descent iterations must be > 0")

    def id_tags(self):
        return sorted({cc.data_configuration.random_effect_type for cc in self.coord_configs.values()
                       if cc.is_random_effect})

    # ------------------------------------------------------------------------------------------------------
    def run(self) -> Dict[str, object]:
        a = self.args
        with Timed("Clean output directories"):
            if not (a.resume and os.path.exists(a.root_output_directory)):
                process_output_dir(a.root_output_directory, a.override_output_directory)
            if a.data_summary_directory and not a.resume:
                process_output_dir(a.data_summary_directory, a.override_output_directory)
        self.logger = PhotonLogger(os.path.join(a.root_output_directory, LOGS), a.logging_level, rank=rank())
        try:
            return self._run()
        finally:
            self.logger.close()

    def _run(self):
        a = self.args
        with Timed("Prepare features"):
            maps = self.prepare_feature_maps()
        with Timed("Read training data"):
            train_paths = resolve_paths(a.input_data_directories, a.input_data_date_range, a.input_data_days_range)
            train, maps = self.read(train_paths, maps)
            self.log(f"training rows: {train.n_rows}; shards: "
                     + ", ".join(f"{s}={m.feature_dimension}" for s, m in maps.items()))
        validation = None
        if a.validation_data_directories:
            with Timed("Read validation data"):
                vpaths = resolve_paths(a.validation_data_directories, a.validation_data_date_range,
                                       a.validation_data_days_range)
                validation, _ = self.read(vpaths, maps)
        with Timed("Validate data"):
            for d in [train] + ([validation] if validation is not None else []):
                sanity_check(a.training_task, d.response, d.offsets, d.weights, d.shards,
                             DataValidationType.parse(a.data_validation))
        stats = None
        if a.data_summary_directory or self.normalization != NormalizationType.NONE:
            with Timed("Calculate statistics for each feature shard"):
                stats = {sid: BasicStatisticalSummary.compute(train.shards[sid], all_reduce=is_dist())
                         for sid in self.shard_configs}
            if a.data_summary_directory and rank() == 0:
                for sid, st in stats.items():
                    d = os.path.join(a.data_summary_directory, sid)
                    os.makedirs(d, exist_ok=True)
                    save_feature_summary(os.path.join(d, "part-00000.avro"), st, maps[sid])
        norm_ctx = {}
        if self.normalization != NormalizationType.NONE:
            shard_ctx = {sid: NormalizationContext.build(self.normalization, st, maps[sid].intercept_index)
                         for sid, st in stats.items()}
            norm_ctx = {cid: shard_ctx[cc.data_configuration.feature_shard_id]
                        for cid, cc in self.coord_configs.items() if not cc.is_random_effect}
        configs = expand_game_configurations(self.coord_configs)
        self.log(f"{len(configs)} optimization configuration(s)")
        est = (GameEstimator(device=a.device, precision=a.precision)
               .set_training_task(a.training_task)
               .set_coordinate_data_configurations({cid: cc.data_configuration
                                                    for cid, cc in self.coord_configs.items()})
               .set_coordinate_update_sequence(self.update_sequence)
               .set_coordinate_descent_iterations(a.coordinate_descent_iterations)
               .set_compute_variance(a.compute_variance)
               .set_warm_start(a.use_warm_start)
               .set_tree_aggregate_depth(a.tree_aggregate_depth)
               .set_coordinate_normalization_contexts(norm_ctx))
        if a.model_input_directory:
            from ..io.model_io import load_game_model
            est.set_initial_model(load_game_model(a.model_input_directory, maps))
        if a.evaluators:
            est.set_validation_evaluators(split_list(a.evaluators))
        if a.checkpoint_directory:
            est.set_checkpoint_directory(a.checkpoint_directory, a.resume)
        with Timed("Fit models"):
            explicit = est.fit(train, validation, configs)
        for i, r in enumerate(explicit):
            if r.evaluations:
                self.log(f"model {i}: " + ", ".join(f"{e.name}={v:.6g}" for e, v in r.evaluations))
        with Timed("Tune hyper-parameters"):
            tuned = self.run_hyperparameter_tuning(est, train, validation, explicit)
        outputs, best = self.select_models(explicit, tuned)
        with Timed("Save models"):
            if rank() == 0:
                self.save_models(maps, outputs, best)
        return {"explicit": explicit, "tuned": tuned, "best": best, "index_maps": maps}

    def run_hyperparameter_tuning(self, est, train, validation, models: List[GameResult]) -> List[GameResult]:
        if validation is None or self.tuning == HyperparameterTuningMode.NONE:
            return []
        fn = GameEstimatorEvaluationFunction(est, models[0].config, train, validation,
                                             self.args.hyper_parameter_tuning_scale)
        evaluator = models[0].evaluations[0][0]
        fn.higher_is_better = evaluator.higher_is_better
        ranges = fn.search_ranges(DoubleRange.parse(self.args.hyper_parameter_tuning_range))
        if self.tuning == HyperparameterTuningMode.BAYESIAN:
            searcher = GaussianProcessSearch(ranges, fn, evaluator.higher_is_better)
        else:
            searcher = RandomSearch(ranges, fn)
        return searcher.find(self.args.hyper_parameter_tuning_iterations, models)

    def select_models(self, explicit, tuned):
        mode = self.output_mode
        outputs = {ModelOutputMode.NONE: [], ModelOutputMode.BEST: [], ModelOutputMode.EXPLICIT: explicit,
                   ModelOutputMode.TUNED: tuned, ModelOutputMode.ALL: explicit + tuned}[mode]
        best = None if mode == ModelOutputMode.NONE else self.select_best_model(explicit + tuned)
        return outputs, best

    def select_best_model(self, models: List[GameResult]) -> Optional[GameResult]:
        best = None
        for r in models:
            if not r.evaluations:
                continue
            if best is None:
                best = r
                continue
            e1, s1 = best.evaluations[0]
            e2, s2 = r.evaluations[0]
            if e1.name != e2.name:
                raise ValueError("Evaluator mismatch while selecting best model")
            # reference reduceOption keeps the LATER model unless the earlier is strictly better
            if not e1.better_than(s1, s2):
                best = r
        if best is None:
            self.log("Could not select best model; missing evaluation results.")
            # without validation data the reference saves nothing under best/; keep the last explicit model so a
            # training run always leaves a usable model
            if models:
                best = models[-1]
        else:
            e, s = best.evaluations[0]
            self.log(f"Best model has {e.name} score of {s} and following config:\n"
                     + optimization_config_to_string(best.config, self.coord_configs))
        return best

    def _save(self, out_dir: str, maps, result: GameResult):
        os.makedirs(out_dir, exist_ok=True)
        with open(os.path.join(out_dir, MODEL_SPEC_DIR), "w") as f:
            f.write(optimization_config_to_string(result.config, self.coord_configs))
        save_game_model(result.model, out_dir, maps, self.args.training_task, result.config,
                        self.args.output_files_limit)

    def save_models(self, maps, outputs: List[GameResult], best: Optional[GameResult]):
        if self.output_mode == ModelOutputMode.NONE:
            return
        root = self.args.root_output_directory
        if best is not None:
            self._save(os.path.join(root, BEST_MODEL_DIR), maps, best)
            self.log("Saved best model")
        for i, r in enumerate(outputs):
            self._save(os.path.join(root, MODELS_DIR, str(i)), maps, r)


def optimization_config_to_string(config, coord_configs=None) -> str:
    """IOUtils.optimizationConfigToString: fixed effects first, then random effects, each by id."""
    def is_re(cid):
        return bool(coord_configs) and cid in coord_configs and coord_configs[cid].is_random_effect
    items = sorted(config.items(), key=lambda kv: (is_re(kv[0]), kv[0]))
    return "".join(f"{cid}:\n{json.dumps(c.to_json(), sort_keys=True)}\n" for cid, c in items)


def main(argv=None) -> int:
    args = parse_args_with_config(build_parser(), argv)
    if "LOCAL_RANK" in os.environ or "RANK" in os.environ:
        from ..parallel.dist import init_distributed, set_allreduce_algo
        set_allreduce_algo(args.allreduce_algo, args.tree_aggregate_depth)
        init_distributed()
    with Timed("Total time in training Driver"):
        GameTrainingDriver(args).run()
    return 0


if __name__ == "__main__":
    sys.exit(main())
