"""Legacy single-GLM training driver (``photon-ml`` CLI).

Reference: ``photon-client/.../Driver.scala:60-740`` with ``Params.scala`` (defaults / validation),
``PhotonMLCmdLineParser.scala`` + ``PhotonOptionNames.scala`` (flag names), ``io/deprecated/GLMSuite.scala``
(Avro / LibSVM input, selected-features file, box-constraint JSON with ``*`` wildcards),
``ModelSelection.scala`` and ``DriverStage.scala``.

Stages: INIT -> PREPROCESSED (read + validate data, optional feature summary / normalization) -> TRAINED (λ path,
descending, warm-started) -> VALIDATED (per-λ metrics, best model by RMSE / log-likelihood / AUROC) ->
DIAGNOSED (HTML + text diagnostic report). Outputs under ``--output-directory``:
``learned-models-text/part-00000`` (``name\\tterm\\tvalue\\tλ``, coefficients sorted descending),
``best-model-text/part-00000``, ``diagnostic.html`` / ``diagnostic.txt``, ``log-message.txt``.
Events (setup, training start/finish, per-λ optimisation log) go to listeners named by ``--event-listeners``.

Usage::

    python -m photon_ml_amd.cli.driver --training-data-directory train/ --validating-data-directory val/ \\
        --output-directory out/ --task LOGISTIC_REGRESSION --regularization-weights 0.1,1,10 --optimizer TRON
"""
from __future__ import annotations

import argparse
import enum
import json
import os
import shutil
import sys
import time
from typing import Dict, List, Optional, Tuple

import numpy as np

from ..constants import DELIMITER, INTERCEPT_KEY, TaskType, split_feature_key
from ..data.matrix import LabeledData
from ..data.validators import DataValidationType, sanity_check
from ..diagnostics.diagnostics import (bootstrap_diagnostic, fitting_diagnostic, validation_diagnostics)
from ..diagnostics.evaluation import evaluate, select_best_model
from ..diagnostics.reporting import build_document
from ..estimators.game_estimator import train_generalized_linear_model
from ..io.data_reader import AvroDataReader, read_libsvm
from ..io.index_map import open_index_map
from ..io.model_io import write_text_models
from ..io.score_io import save_feature_summary
from ..normalization.context import NormalizationContext, NormalizationType
from ..optimization.config import OptimizerType, RegularizationContext, RegularizationType
from ..stat.summary import BasicStatisticalSummary
from ..utils.logging_utils import EventEmitter, PhotonLogger
from .params import add_config_arguments, parse_args_with_config, parse_bool, split_list

LEARNED_MODELS_TEXT = "learned-models-text"
BEST_MODEL_TEXT = "best-model-text"
WILDCARD = "*"


class DriverStage(enum.IntEnum):
    INIT = 0
    PREPROCESSED = 1
    TRAINED = 2
    VALIDATED = 3
    DIAGNOSED = 4


class DiagnosticMode(str, enum.Enum):
    NONE = "NONE"
    TRAIN = "TRAIN"
    VALIDATE = "VALIDATE"
    ALL = "ALL"


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="photon-ml", description="Photon-ML legacy GLM training driver")
    p.add_argument("--training-data-directory", required=True)
    p.add_argument("--validating-data-directory")
    p.add_argument("--output-directory", required=True)
    p.add_argument("--task", required=True)
    p.add_argument("--job-name", default="Photon-ML-Training")
    p.add_argument("--regularization-weights", default="10")
    p.add_argument("--intercept", type=parse_bool, default=True)
    p.add_argument("--num-iterations", type=int, default=80)
    p.add_argument("--convergence-tolerance", type=float, default=1e-6)
    p.add_argument("--optimizer", default="LBFGS")
    p.add_argument("--regularization-type", default="L2")
    p.add_argument("--elastic-net-alpha", type=float)
    p.add_argument("--optimization-tracker", type=parse_bool, default=True)
    p.add_argument("--validate-per-iteration", type=parse_bool, default=False)
    p.add_argument("--min-partitions", type=int, default=1)
    p.add_argument("--kryo", type=parse_bool, default=True)  # accepted for compatibility (no JVM)
    p.add_argument("--format", default="RESPONSE_PREDICTION", help="field names: RESPONSE_PREDICTION | TRAINING_EXAMPLE")
    p.add_argument("--summarization-output-dir")
    p.add_argument("--normalization-type", default="NONE")
    p.add_argument("--coefficient-box-constraints")
    p.add_argument("--data-validation-type", default="VALIDATE_FULL")
    p.add_argument("--tree-aggregate-depth", type=int, default=1,
                   help="reduction depth of the reference's treeAggregate: >= 2 selects RCCL's tree all-reduce "
                        "(unless --allreduce-algo says otherwise), 1 leaves the choice to RCCL")
    p.add_argument("--allreduce-algo", choices=["auto", "ring", "tree"], default=None,
                   help="RCCL all-reduce algorithm of the gradient reduction (NCCL_ALGO); default: from "
                        "--tree-aggregate-depth")
    p.add_argument("--diagnostic-mode", default="NONE")
    p.add_argument("--training-diagnostics", type=parse_bool, default=None,
                   help="deprecated alias: true -> --diagnostic-mode ALL")
    p.add_argument("--selected-features-file")
    p.add_argument("--offheap-indexmap-dir")
    p.add_argument("--offheap-indexmap-num-partitions", type=int)
    p.add_argument("--delete-output-dirs-if-exist", type=parse_bool, default=False)
    p.add_argument("--event-listeners", default="")
    p.add_argument("--input-file-format", default="AVRO", choices=["AVRO", "LIBSVM"])
    p.add_argument("--feature-dimension", type=int, default=-1)
    p.add_argument("--use-warm-start", type=parse_bool, default=True)
    p.add_argument("--device", default=None)
    p.add_argument("--precision", default="f64", choices=["bf16", "f32", "f64"])
    p.add_argument("--seed", type=int, default=0)
    add_config_arguments(p)
    return p


def validate_params(a) -> None:
    """Params.validate (Params.scala:189-222)."""
    msgs = []
    reg = RegularizationType.parse(a.regularization_type)
    opt = OptimizerType.parse(a.optimizer)
    norm = NormalizationType.parse(a.normalization_type)
    diag = DiagnosticMode(a.diagnostic_mode.upper())
    if reg in (RegularizationType.L1, RegularizationType.ELASTIC_NET) and opt == OptimizerType.TRON:
        msgs.append(f"Combination of ({reg.value}, {opt.value}) is not allowed.")
    if a.coefficient_box_constraints and norm != NormalizationType.NONE:
        msgs.append("Normalization and box constraints should not be used together since we cannot guarantee the "
                    "satisfaction of the coefficient constraints after normalization.")
    if norm == NormalizationType.STANDARDIZATION and not a.intercept:
        msgs.append(f"Intercept must be used to enable feature standardization. Normalization type: {norm.value}, "
                    f"add intercept: {a.intercept}.")
    if a.validating_data_directory is None and diag in (DiagnosticMode.VALIDATE, DiagnosticMode.ALL):
        msgs.append(f"Diagnostic mode cannot be {diag.value} when the validate directory is not specified.")
    if msgs:
        raise ValueError("\n".join(msgs))


def constraint_map_from_json(text: Optional[str], index_map) -> Optional[Dict[int, Tuple[float, float]]]:
    """GLMSuite.createConstraintFeatureMap: JSON list of {name, term, lowerBound?, upperBound?}; ``*`` wildcards."""
    if not text:
        return None
    entries = json.loads(text)
    keys = index_map.keys_in_order()
    out: Dict[int, Tuple[float, float]] = {}
    for e in entries:
        if "name" not in e or "term" not in e:
            raise ValueError(f"Each map in the constraint map is expected to have the feature name field specified. "
                             f"The malformed map was [{e}]")
        name, term = e["name"], e["term"]
        lo = float(e.get("lowerBound", -np.inf))
        hi = float(e.get("upperBound", np.inf))
        if lo == -np.inf and hi == np.inf:
            raise ValueError(f"The lower and upper bound are respectively -Inf and +Inf for the feature with name "
                             f"[{name}] and term [{term}]. This is an invalid constraint specification.")
        if not lo < hi:
            raise ValueError(f"The lower bound [{lo}] is incorrectly specified as greater than the upper bound [{hi}] "
                             f"for the feature with name [{name}] and term [{term}].")
        if name == WILDCARD:
            if term != WILDCARD:
                raise ValueError("Wildcard in the feature name alone is not supported")
            if out:
                raise ValueError("Potentially conflicting constraints specified: a full wildcard must be the only "
                                 "constraint")
            for j, k in enumerate(keys):
                if k is not None and k != INTERCEPT_KEY:
                    out[j] = (lo, hi)
            continue
        if term == WILDCARD:
            targets = [j for j, k in enumerate(keys) if k is not None and k.startswith(name + DELIMITER)]
        else:
            j = index_map.get_index(name + DELIMITER + term)
            targets = [j] if j >= 0 else []
        for j in targets:
            if j in out:
                raise ValueError(f"Please avoid specifying potentially conflicting bounds (feature {keys[j]!r})")
            out[j] = (lo, hi)
    return out or None


class Driver:
    def __init__(self, args, seed: Optional[int] = None):
        validate_params(args)
        self.a = args
        self.seed = args.seed if seed is None else seed
        self.task = TaskType.parse(args.task)
        self.stage = DriverStage.INIT
        self.stage_history: List[DriverStage] = []
        self.reg = RegularizationContext(args.regularization_type, args.elastic_net_alpha)
        self.diag = DiagnosticMode(args.diagnostic_mode.upper())
        if args.training_diagnostics:
            self.diag = DiagnosticMode.ALL if args.validating_data_directory else DiagnosticMode.TRAIN
        self.events = EventEmitter()
        for cls in split_list([args.event_listeners]):
            self.events.register_by_name(cls)
        self.logger: Optional[PhotonLogger] = None
        self.train_data: Optional[LabeledData] = None
        self.validation_data: Optional[LabeledData] = None
        self.index_map = None
        self.summary = None
        self.normalization: Optional[NormalizationContext] = None
        self.lambda_models: List[Tuple[float, object]] = []
        self.trackers = {}
        self.per_model_metrics: Dict[float, dict] = {}
        self.best: Optional[Tuple[float, object]] = None
        self.model_reports = []

    # --------------------------------------------------------------------------------------------------
    def _update_stage(self, s: DriverStage):
        self.stage_history.append(self.stage)
        self.stage = s

    def _assert_stage(self, s: DriverStage):
        if self.stage != s:
            raise RuntimeError(f"Expecting driver stage {s.name} but actually it is {self.stage.name}")

    def log(self, msg):
        if self.logger is not None:
            self.logger.info(msg)

    def _process_output_dir(self, d):
        if os.path.exists(d):
            if not self.a.delete_output_dirs_if_exist:
                raise FileExistsError(f"Output directory {d} already exists")
            shutil.rmtree(d)

    def run(self):
        a = self.a
        self._process_output_dir(a.output_directory)
        if a.summarization_output_dir:
            self._process_output_dir(a.summarization_output_dir)
        os.makedirs(a.output_directory, exist_ok=True)
        self.logger = PhotonLogger(a.output_directory, "INFO", name="photon_ml_amd.driver")
        self.events.emit("PhotonSetupEvent", params=vars(a))
        t0 = time.time()
        self.events.emit("TrainingStartEvent", time=t0)
        try:
            self._assert_stage(DriverStage.INIT)
            self.preprocess()
            self._update_stage(DriverStage.PREPROCESSED)
            self.train()
            self._update_stage(DriverStage.TRAINED)
            if self.validation_data is not None:
                self.validate()
                self._update_stage(DriverStage.VALIDATED)
            else:
                for lam, tr in self.trackers.items():
                    self.events.emit("PhotonOptimizationLogEvent", regularization_weight=lam, tracker=str(tr))
            if self.diag != DiagnosticMode.NONE:
                self.diagnose()
                self._update_stage(DriverStage.DIAGNOSED)
            write_text_models(self.lambda_models, self.index_map,
                              os.path.join(a.output_directory, LEARNED_MODELS_TEXT, "part-00000"))
            self.log(f"total time elapsed: {time.time() - t0:.3f}(s)")
            self.events.emit("TrainingFinishEvent", time=time.time())
        finally:
            self.events.close()
            self.logger.close()
        return self

    # --------------------------------------------------------------------------------------------------
    def _read(self, path: str, index_map=None) -> Tuple[LabeledData, object]:
        a = self.a
        if a.input_file_format == "LIBSVM":
            dim = a.feature_dimension if a.feature_dimension > 0 else (
                None if index_map is None else index_map.feature_dimension - (1 if a.intercept else 0))
            data, im = read_libsvm(path, dim, add_intercept=a.intercept,
                                   binarize_labels=self.task in (TaskType.LOGISTIC_REGRESSION,
                                                                 TaskType.SMOOTHED_HINGE_LOSS_LINEAR_SVM))
            return data, index_map or im
        reader = AvroDataReader()
        if a.format.upper() == "TRAINING_EXAMPLE":
            reader.columns.response = "label"
        if index_map is None and a.offheap_indexmap_dir:
            index_map = open_index_map(a.offheap_indexmap_dir, "global", a.offheap_indexmap_num_partitions or 1)
        if index_map is None and a.selected_features_file:
            from ..io.avro import avro_files, read_records
            keys = set()
            for f in avro_files(a.selected_features_file):
                keys.update(r["name"] + DELIMITER + (r.get("term") or "") for r in read_records(f)[1])
            from ..io.index_map import DefaultIndexMap
            index_map = DefaultIndexMap.from_keys(sorted(keys), add_intercept=a.intercept)
        return reader.read_labeled(path, index_map, ("features",), a.intercept)

    def preprocess(self):
        a = self.a
        t = time.time()
        if a.selected_features_file and not os.path.exists(a.selected_features_file):
            raise FileNotFoundError(f"Could not find [{a.selected_features_file}]. Check that the file exists")
        self.train_data, self.index_map = self._read(a.training_data_directory)
        if self.train_data.n_rows == 0:
            raise ValueError("No training data found.")
        self.log(f"Number of training data points: {self.train_data.n_rows}, number of features including "
                 f"intercept: {self.train_data.n_features}")
        sanity_check(self.task, self.train_data.y, self.train_data.offsets, self.train_data.weights,
                     {"features": self.train_data.x}, a.data_validation_type)
        if a.validating_data_directory:
            self.validation_data, _ = self._read(a.validating_data_directory, self.index_map)
            sanity_check(self.task, self.validation_data.y, self.validation_data.offsets, self.validation_data.weights,
                         {"features": self.validation_data.x}, a.data_validation_type)
        norm = NormalizationType.parse(a.normalization_type)
        if a.summarization_output_dir or norm != NormalizationType.NONE:
            self.summary = BasicStatisticalSummary.compute(self.train_data.x)
            if a.summarization_output_dir:
                os.makedirs(a.summarization_output_dir, exist_ok=True)
                save_feature_summary(os.path.join(a.summarization_output_dir, "part-00000.avro"), self.summary,
                                     self.index_map)
            self.normalization = NormalizationContext.build(norm, self.summary, self.index_map.intercept_index)
        self.log(f"preprocessing data finished, time elapsed: {time.time() - t:.3f}(s)")

    def _train(self, data: LabeledData, warm: Optional[dict] = None):
        a = self.a
        res = train_generalized_linear_model(
            data, self.task, a.optimizer, self.reg, [float(x) for x in split_list([a.regularization_weights])],
            self.normalization, a.num_iterations, a.convergence_tolerance,
            constraint_map_from_json(a.coefficient_box_constraints, self.index_map), warm, a.use_warm_start,
            device=a.device, precision=a.precision)
        return res

    def train(self):
        t = time.time()
        res = self._train(self.train_data)
        self.lambda_models = [(lam, m) for lam, m, _ in res]
        self.trackers = {lam: tr for lam, _, tr in res}
        self.log(f"model training finished, time elapsed: {time.time() - t:.3f}(s)")
        for lam, tr in self.trackers.items():
            self.log(f"model with regularization weight {lam}: {tr}")

    def validate(self):
        for lam, m in self.lambda_models:
            met = evaluate(m, self.validation_data)
            self.per_model_metrics[lam] = met
            self.log(f"Model with lambda = {lam}:\n" + "\n".join(f"    Metric: [{k}] value: {v}"
                                                              for k, v in sorted(met.items())))
            self.events.emit("PhotonOptimizationLogEvent", regularization_weight=lam,
                             tracker=str(self.trackers.get(lam)), final_metrics=met)
        self.best = select_best_model(self.task, self.lambda_models, self.per_model_metrics)
        self.log(f"Regularization weight of the best model is: {self.best[0]}")
        write_text_models([self.best], self.index_map, os.path.join(self.a.output_directory, BEST_MODEL_TEXT,
                                                                   "part-00000"))

    def _train_func(self, data, warm):
        return [(lam, m) for lam, m, _ in self._train(data, warm)]

    def diagnose(self):
        t = time.time()
        models = dict(self.lambda_models)
        fit, boot = {}, {}
        if self.diag in (DiagnosticMode.TRAIN, DiagnosticMode.ALL):
            fit = fitting_diagnostic(self._train_func, models, self.train_data, self.seed)
            boot = bootstrap_diagnostic(self._train_func, models, self.train_data, self.index_map, self.summary,
                                        seed=self.seed)
        reports = []
        for lam, m in self.lambda_models:
            if self.diag in (DiagnosticMode.VALIDATE, DiagnosticMode.ALL):
                rep = validation_diagnostics(m, lam, self.validation_data, self.index_map, self.summary,
                                             self.per_model_metrics.get(lam), self.seed)
            else:
                from ..diagnostics.diagnostics import ModelDiagnosticReport
                rep = ModelDiagnosticReport(m, lam, f"{type(m).__name__} @ lambda = {lam}",
                                            self.per_model_metrics.get(lam, {}), self.summary)
            rep.fit_report = fit.get(lam)
            rep.bootstrap_report = boot.get(lam)
            reports.append(rep)
        self.model_reports = reports
        doc = build_document(f"Photon-ML diagnostics: {self.a.job_name}", reports,
                             {k: v for k, v in vars(self.a).items() if v is not None}, self.index_map, self.summary)
        with open(os.path.join(self.a.output_directory, "diagnostic.html"), "w") as f:
            f.write(doc.to_html())
        with open(os.path.join(self.a.output_directory, "diagnostic.txt"), "w") as f:
            f.write(doc.to_text())
        self.log(f"Total diagnostic time: {time.time() - t:.3f} (s)")


def read_text_model(path: str) -> Dict[float, Dict[Tuple[str, str], float]]:
    """Parse ``learned-models-text`` output back into {λ: {(name, term): value}}."""
    out: Dict[float, Dict[Tuple[str, str], float]] = {}
    files = [os.path.join(path, f) for f in sorted(os.listdir(path))] if os.path.isdir(path) else [path]
    for fn in files:
        with open(fn) as f:
            for line in f:
                n, t, v, lam = line.rstrip("\n").split("\t")
                out.setdefault(float(lam), {})[(n, t)] = float(v)
    return out


def main(argv=None) -> int:
    args = parse_args_with_config(build_parser(), argv)
    from ..parallel.dist import set_allreduce_algo
    set_allreduce_algo(args.allreduce_algo, args.tree_aggregate_depth)
    Driver(args).run()
    return 0


if __name__ == "__main__":
    sys.exit(main())
