"""Score and feature-statistics output (``ScoringResultAvro``, ``FeatureSummarizationResultAvro``).

Reference: ``photon-client/.../data/avro/ScoreProcessingUtils.scala:29-88`` (predictionScore = score + offset,
modelId default "N/A", optional uid/label/weight/metadataMap; output coalesced to a file limit) and
``ModelProcessingUtils.scala:573-644`` (feature statistics: max, min, mean, normL1, normL2, numNonzeros,
variance per feature).
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import numpy as np

from ..constants import split_feature_key
from .avro import FEATURE_SUMMARY, SCORING_RESULT, read_records, write_records, avro_files


def save_scores(out_dir: str, scores: np.ndarray, offsets: np.ndarray, labels: Optional[np.ndarray] = None,
                weights: Optional[np.ndarray] = None, uids: Optional[np.ndarray] = None, model_id: str = "N/A",
                metadata: Optional[Dict[str, np.ndarray]] = None, file_limit: Optional[int] = None,
                records_per_file: int = 1_000_000):
    n = len(scores)
    pred = np.asarray(scores, dtype=np.float64) + np.asarray(offsets, dtype=np.float64)
    recs = []
    for i in range(n):
        md = None
        if metadata:
            md = {k: str(v[i]) for k, v in metadata.items() if v[i] is not None and str(v[i]) != ""}
        recs.append({"uid": None if uids is None or uids[i] is None else str(uids[i]),
                     "label": None if labels is None or np.isnan(labels[i]) else float(labels[i]),
                     "modelId": model_id, "predictionScore": float(pred[i]),
                     "weight": None if weights is None else float(weights[i]), "metadataMap": md or None})
    n_files = max(1, (n + records_per_file - 1) // records_per_file)
    if file_limit is not None:
        n_files = max(1, min(n_files, file_limit))
    per = (n + n_files - 1) // n_files if n else 0
    os.makedirs(out_dir, exist_ok=True)
    for i in range(n_files):
        write_records(os.path.join(out_dir, f"part-{i:05d}.avro"), SCORING_RESULT, recs[i * per:(i + 1) * per])


def load_scores(path) -> list:
    out = []
    for f in avro_files(path):
        out.extend(read_records(f)[1])
    return out


def save_feature_summary(path: str, summary, index_map):
    """One FeatureSummarizationResultAvro per feature (intercept excluded, as in the reference)."""
    recs = []
    for j in range(index_map.feature_dimension):
        key = index_map.get_feature_name(j)
        if key is None:
            continue
        name, term = split_feature_key(key)
        if name == "(INTERCEPT)":
            continue
        recs.append({"featureName": name, "featureTerm": term, "metrics": {
            "max": float(summary.max[j]), "min": float(summary.min[j]), "mean": float(summary.mean[j]),
            "normL1": float(summary.norm_l1[j]), "normL2": float(summary.norm_l2[j]),
            "numNonzeros": float(summary.num_nonzeros[j]), "variance": float(summary.variance[j])}})
    write_records(path, FEATURE_SUMMARY, recs)
