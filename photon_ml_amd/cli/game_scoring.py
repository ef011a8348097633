"""GAME scoring driver (command line).

Reference: ``photon-client/.../cli/game/scoring/GameScoringDriver.scala:49-300``: process the output directory,
prepare feature maps, read the data, validate, load the GAME model (``model-metadata.json`` + Avro coefficients),
score with ``GameTransformer`` (optionally evaluating), and write ``<root>/scores/part-*.avro``
(``ScoringResultAvro``; predictionScore = model score + offset, ``modelId`` from ``--model-id``).

Multi-GPU: each rank scores its slice of the input files (rank r > 0 writes under ``scores/rank-<r>/``); evaluation
metrics are computed on rank-local data and logged per rank.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

from ..data.validators import DataValidationType, sanity_check
from ..estimators.game_estimator import GameTransformer
from ..io.model_io import load_game_model, load_model_task
from ..io.score_io import save_scores
from ..models.game import RandomEffectModel
from ..parallel.dist import rank
from ..utils.logging_utils import PhotonLogger
from ..utils.timing import Timed
from .game_training import GameDriverBase, add_common_arguments, process_output_dir, resolve_paths
from .params import parse_args_with_config, parse_bool, split_list

SCORES_DIR = "scores"
DEFAULT_APPLICATION_NAME = "GAME-Scoring"


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="game-scoring", description=__doc__.split("\n")[0])
    add_common_arguments(p)
    p.add_argument("--model-input-directory", required=True)
    p.add_argument("--model-id", default="N/A")
    p.add_argument("--log-data-and-model-stats", type=parse_bool, default=False)
    p.add_argument("--spill-scores-to-disk", type=parse_bool, default=False,
                   help="score the rows in chunks straight into a memory-mapped score file under the output "
                        "directory instead of keeping every score resident (the reference's MEMORY_AND_DISK "
                        "persistence of the scores RDD); removed after the scores are written")
    p.add_argument("--spill-chunk-rows", type=int, default=1 << 24,
                   help="rows scored per device chunk with --spill-scores-to-disk")
    return p


class GameScoringDriver(GameDriverBase):
    def __init__(self, args):
        super().__init__(args)
        self.model = None
        self._tags = []

    def id_tags(self):
        return self._tags

    def run(self):
        a = self.args
        process_output_dir(a.root_output_directory, a.override_output_directory)
        self.logger = PhotonLogger(a.root_output_directory, a.logging_level, rank=rank())
        try:
            return self._run()
        finally:
            self.logger.close()

    def _run(self):
        a = self.args
        with Timed("Prepare features"):
            maps = self.prepare_feature_maps()
        # without explicit maps the reader builds them from the scoring data (as readMerged does); model
        # coefficients of features absent from the data are dropped on load, which leaves every score unchanged
        # random-effect id tags come from the model directory layout (random-effect/<cid>/id-info)
        re_dir = os.path.join(a.model_input_directory, "random-effect")
        if os.path.isdir(re_dir):
            for cid in sorted(os.listdir(re_dir)):
                info = os.path.join(re_dir, cid, "id-info")
                if os.path.exists(info):
                    self._tags.append(open(info).read().split()[0])
        self._tags = sorted(set(self._tags))
        with Timed("Read data"):
            paths = resolve_paths(a.input_data_directories, a.input_data_date_range, a.input_data_days_range)
            data, maps = self.read(paths, maps)
        with Timed("Validate data"):
            sanity_check("LINEAR_REGRESSION", data.response, data.offsets, data.weights, data.shards,
                         DataValidationType.parse(a.data_validation), for_training=bool(a.evaluators))
        with Timed("Load model"):
            self.model = load_game_model(a.model_input_directory, maps)
            self.log(f"model task {load_model_task(a.model_input_directory).value}: {self.model}")
        if a.log_data_and_model_stats:
            for cid, m in self.model:
                if isinstance(m, RandomEffectModel):
                    self.log(f"{cid}: {m.n_entities} entities, {len(m.keys)} non-zero coefficients")
            self.log(f"data: {data.n_rows} rows")
        with Timed("Score data"):
            tr = GameTransformer(self.model, split_list(a.evaluators) if a.evaluators else None,
                                 device=a.device or None)
            self.scoring_device = tr.device
            self.log(f"scoring on {tr.device}")
            spill = None
            if a.spill_scores_to_disk:
                spill = os.path.join(a.root_output_directory, f".scores-spill-{rank():05d}.npy")
                scores, evals = tr.transform_spilled(data, spill, a.spill_chunk_rows)
            else:
                scores, evals = tr.transform(data)
        if evals:
            for e, v in evals:
                self.log(f"evaluation {e.name}: {v}")
        with Timed("Save scores"):
            out = os.path.join(a.root_output_directory, SCORES_DIR)
            if rank() > 0:
                out = os.path.join(out, f"rank-{rank():05d}")
            has_label = not np.all(np.isnan(data.response))
            save_scores(out, scores.cpu().numpy(), data.offsets, data.response if has_label else None,
                        data.weights, data.raw_uids, a.model_id, data.id_tags or None, a.output_files_limit)
        if spill is not None:
            os.remove(spill)      # POSIX: the mapping behind the returned scores stays valid until released
        return {"scores": scores, "evaluations": evals, "data": data}


def main(argv=None) -> int:
    args = parse_args_with_config(build_parser(), argv)
    if "LOCAL_RANK" in os.environ or "RANK" in os.environ:
        from ..parallel.dist import init_distributed
        init_distributed()
    with Timed("Total time in scoring Driver"):
        GameScoringDriver(args).run()
    return 0


if __name__ == "__main__":
    sys.exit(main())
