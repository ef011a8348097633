"""Python face of the native Avro codec (``io/csrc/avro_codec.cpp``) plus the Photon Avro schemas.

Schemas are the reference's (``photon-avro-schemas/src/main/avro/*.avsc``) re-declared as JSON: training examples,
``BayesianLinearModelAvro`` (model coefficients), ``ScoringResultAvro`` and ``FeatureSummarizationResultAvro``.
"""
from __future__ import annotations

import importlib.util
import json
import os
from typing import Iterable, List, Optional, Sequence

from ..ops.build import StaleLibraryError, expected_id, verified_path

_MOD = None


def native():
    global _MOD
    if _MOD is None:
        path = verified_path("cpp", "avro")       # stale builds are rebuilt or refused (ops/build.py build ids)
        spec = importlib.util.spec_from_file_location("libpml_avro", str(path))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        if mod.build_id() != expected_id("cpp", "avro"):
            raise StaleLibraryError(f"{path}: loaded build id {mod.build_id()} != the tree's sources")
        _MOD = mod
    return _MOD


NAME_TERM_VALUE = {
    "type": "record", "name": "NameTermValueAvro", "namespace": "com.linkedin.photon.ml.avro.generated",
    "doc": "A tuple of name, term and value. Used as feature or model coefficient",
    "fields": [{"name": "name", "type": "string"}, {"name": "term", "type": "string"},
               {"name": "value", "type": "double"}],
}

BAYESIAN_LINEAR_MODEL = {
    "type": "record", "name": "BayesianLinearModelAvro", "namespace": "com.linkedin.photon.ml.avro.generated",
    "doc": "a generic schema to describe a Bayesian linear model with means and variances",
    "fields": [
        {"name": "modelId", "type": "string"},
        {"name": "modelClass", "type": "string", "default": None,
         "doc": "The fully-qualified class name of enclosing GLM model class."},
        {"name": "means", "type": {"type": "array", "items": NAME_TERM_VALUE}},
        {"name": "variances", "type": ["null", {"type": "array", "items": "NameTermValueAvro"}], "default": None},
        {"name": "lossFunction", "type": ["null", "string"], "default": None},
    ],
}

FEATURE = {"type": "record", "name": "FeatureAvro", "namespace": "com.linkedin.photon.avro.generated",
           "fields": [{"name": "name", "type": "string"}, {"name": "term", "type": "string"},
                      {"name": "value", "type": "double"}]}

TRAINING_EXAMPLE = {
    "type": "record", "name": "TrainingExampleAvro", "namespace": "com.linkedin.photon.avro.generated",
    "fields": [
        {"name": "uid", "type": ["null", "string"], "default": None},
        {"name": "label", "type": "double"},
        {"name": "features", "type": {"type": "array", "items": FEATURE}},
        {"name": "metadataMap", "type": ["null", {"type": "map", "values": "string"}], "default": None},
        {"name": "weight", "type": ["null", "double"], "default": None},
        {"name": "offset", "type": ["null", "double"], "default": None},
    ],
}

SCORING_RESULT = {
    "type": "record", "name": "ScoringResultAvro", "namespace": "com.linkedin.photon.avro.generated",
    "fields": [
        {"name": "uid", "type": ["null", "string"], "default": None},
        {"name": "label", "type": ["null", "double"], "default": None},
        {"name": "modelId", "type": "string"},
        {"name": "predictionScore", "type": "double"},
        {"name": "weight", "type": ["null", "double"], "default": None},
        {"name": "metadataMap", "type": ["null", {"type": "map", "values": "string"}], "default": None},
    ],
}

LATENT_FACTOR = {
    "type": "record", "name": "LatentFactorAvro", "namespace": "com.linkedin.photon.avro.generated",
    "doc": "latent factor of a matrix-factorization model (schema parity only: the reference has no MF training)",
    "fields": [{"name": "effectId", "type": "string"},
               {"name": "latentFactor", "type": {"type": "array", "items": "double"}}],
}

FEATURE_SUMMARY = {
    "type": "record", "name": "FeatureSummarizationResultAvro", "namespace": "com.linkedin.photon.avro.generated",
    "fields": [{"name": "featureName", "type": "string"}, {"name": "featureTerm", "type": "string"},
               {"name": "metrics", "type": {"type": "map", "values": "double"}}],
}


def read_records(path: str):
    """Return (schema dict, list of records) of one OCF file."""
    schema_json, recs, _codec = native().read_ocf(str(path))
    return json.loads(schema_json), recs


def read_records_many(paths: Iterable[str]) -> List[dict]:
    out = []
    for p in paths:
        out.extend(read_records(p)[1])
    return out


def write_records(path: str, schema, records: Sequence[dict], codec: str = "deflate", block_records: int = 4096):
    sj = schema if isinstance(schema, str) else json.dumps(schema)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    native().write_ocf(str(path), sj, list(records), codec, block_records)


def avro_files(path_or_dir) -> List[str]:
    """Expand a file or directory (recursively) into the list of ``*.avro`` files, sorted."""
    paths = path_or_dir if isinstance(path_or_dir, (list, tuple)) else [path_or_dir]
    out = []
    for p in paths:
        p = str(p)
        if os.path.isdir(p):
            for root, _dirs, files in os.walk(p):
                out.extend(os.path.join(root, f) for f in files if f.endswith(".avro"))
        elif os.path.exists(p):
            out.append(p)
    return sorted(out)
