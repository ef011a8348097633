"""GAME block coordinate descent.

Reference: ``photon-lib/.../algorithm/CoordinateDescent.scala:37-385``:
  * initial model: zero coefficients per coordinate (or a given GAME model);
  * per sweep, for each coordinate in the update sequence: partial = full - own (only when there is more than one
    coordinate), update the coordinate on offsets + partial, rescore, full = full - old + new;
  * after each coordinate: (debug) training objective = training-loss evaluator + regularisation, and validation
    scores updated incrementally and evaluated;
  * best-model selection with the FIRST validation evaluator, compared after each full sweep.
Scores are aligned N-length device tensors, so the score algebra is elementwise.
"""
from __future__ import annotations

import logging
import time
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..models.game import GameModel
from ..utils.timing import Timed

log = logging.getLogger(__name__)


class CoordinateDescent:
    def __init__(self, coordinates: "OrderedDict[str, object]", training_loss_evaluator=None,
                 validation_data=None, validation_evaluators: Sequence = (), score_device=None,
                 event_callback=None):
        self.coordinates = OrderedDict(coordinates)
        self.training_loss_evaluator = training_loss_evaluator
        self.validation_data = validation_data
        self.validation_evaluators = list(validation_evaluators)
        self.score_device = score_device
        self.event_callback = event_callback
        self.history: List[dict] = []

    def _dev(self, t: torch.Tensor) -> torch.Tensor:
        return t if self.score_device is None else t.to(self.score_device)

    def _score_validation(self, cid, model, device):
        coord = self.coordinates[cid]
        if hasattr(coord, "score_validation"):  # entity-sharded coordinates route validation rows to owners
            return coord.score_validation(model, self.validation_data)
        return model.score(self.validation_data, device)

    def run(self, iterations: int, initial_model: Optional[GameModel] = None, checkpointer=None,
            tag: str = "") -> Tuple[GameModel, Optional[list]]:
        """``checkpointer`` (:class:`photon_ml_amd.utils.checkpoint.Checkpointer`): save the state after every
        coordinate update and, when a state with the same ``tag`` exists, resume from the coordinate after the
        last one saved (scores are recomputed from the restored model)."""
        if iterations <= 0:
            raise ValueError(f"Number of coordinate descent iterations must be greater than 0: {iterations}")
        start_it, start_c = 0, 0
        resumed = None
        if checkpointer is not None:
            st = checkpointer.load_cd()
            if st is not None and st.get("tag", "") == tag:
                resumed = st
                initial_model = st["model"]
                start_it, start_c = st["iteration"], st["next"]
                self.history = list(st["history"])
                log.info("resuming coordinate descent at iteration %d, coordinate %d", start_it, start_c)
        if initial_model is None:
            initial_model = GameModel(OrderedDict((cid, c.initialize_model()) for cid, c in self.coordinates.items()))
        for cid in self.coordinates:
            if initial_model.get(cid) is None:
                raise ValueError(f"Model with coordinateId {cid} is expected but not found from the initial GAME model")
        model = initial_model
        scores = {cid: self._dev(c.score(model.get(cid))) for cid, c in self.coordinates.items()}
        full = sum(scores.values())
        reg_terms = {cid: c.regularization_term_value(model.get(cid)) for cid, c in self.coordinates.items()}
        val_scores, val_full = None, None
        if self.validation_data is not None:
            val_scores = {cid: self._dev(self._score_validation(cid, model.get(cid), full.device))
                          for cid in self.coordinates}
            val_full = sum(val_scores.values())
        best_model, best_evals = None, None
        if resumed is not None and resumed["best_model"] is not None and resumed["best_evals"]:
            by_name = {e.name: e for e in self.validation_evaluators}
            best_model = resumed["best_model"]
            best_evals = [(by_name[n], v) for n, v in resumed["best_evals"] if n in by_name] or None
        cids = list(self.coordinates)
        evaluations = None
        for it in range(start_it, iterations):
            with Timed(f"Coordinate descent iteration {it}", log):
                if it > start_it or start_c == 0:
                    evaluations = None
                for ci, (cid, coord) in enumerate(self.coordinates.items()):
                    if it == start_it and ci < start_c:
                        continue
                    t0 = time.time()
                    old = model.get(cid)
                    with Timed(f"Update coordinate {cid}", log):
                        if len(scores) > 1:
                            partial = full - scores[cid]
                            new = coord.update_model(old, partial)
                        else:
                            new = coord.update_model(old)
                    model = model.updated(cid, new)
                    new_scores = self._dev(coord.score(new))
                    full = full - scores[cid] + new_scores
                    scores[cid] = new_scores
                    reg_terms[cid] = coord.regularization_term_value(new)
                    rec = {"iteration": it, "coordinate": cid, "seconds": time.time() - t0}
                    if self.training_loss_evaluator is not None:
                        loss = self.training_loss_evaluator.evaluate(full)
                        rec["training_loss"] = loss
                        rec["objective"] = loss + sum(reg_terms.values())
                    if self.validation_data is not None:
                        vs = self._dev(self._score_validation(cid, new, full.device))
                        val_full = val_full - val_scores[cid] + vs
                        val_scores[cid] = vs
                        evaluations = [(e, e.evaluate(val_full)) for e in self.validation_evaluators]
                        rec["validation"] = {e.name: v for e, v in evaluations}
                        for e, v in evaluations:
                            log.info("Evaluation metric computed with %s after updating coordinateId %s at "
                                     "iteration %d is %s", e.name, cid, it, v)
                    self.history.append(rec)
                    if self.event_callback is not None:
                        self.event_callback(rec)
                    last = ci == len(cids) - 1
                    if last and evaluations:
                        e0, v0 = evaluations[0]
                        if best_evals is None or e0.better_than(v0, best_evals[0][1]):
                            best_model, best_evals = model, evaluations
                    if checkpointer is not None:
                        nxt_it, nxt_c = (it + 1, 0) if last else (it, ci + 1)
                        checkpointer.save_cd(model, nxt_it, nxt_c, best_model,
                                             None if best_evals is None else [(e.name, v) for e, v in best_evals],
                                             self.history, tag)
        if self.validation_data is not None and evaluations is None and best_evals is None:
            # resumed exactly at the end of the last sweep: re-evaluate the restored model
            evaluations = [(e, e.evaluate(val_full)) for e in self.validation_evaluators]
            best_model, best_evals = model, evaluations
        return (best_model if best_model is not None else model), best_evals
