"""Command-line parameter parsing shared by the drivers (reference flag names, ``k=v`` DSL).

Reference: ``photon-client/.../io/scopt/ScoptParameter.scala`` (param name -> ``--param-name``),
``ScoptParserHelpers.scala:34-457`` (DSL keys: ``name``, ``feature.bags`` (| separated), ``intercept``,
``random.effect.type``, ``feature.shard``, ``min.partitions``, ``active.data.bound``, ``passive.data.bound``,
``features.to.samples.ratio``, ``optimizer``, ``max.iter``, ``tolerance``, ``regularization``, ``reg.alpha``,
``reg.weights`` (| separated), ``down.sampling.rate``), ``CLI/io/CoordinateConfiguration.scala`` (λ grid expanded
descending), ``CLI/io/ModelOutputMode.scala``, ``CLI/util/{DateRange,DaysRange}.scala`` and
``CLI/util/IOUtils.scala`` (daily ``yyyy/MM/dd`` input directories).
"""
from __future__ import annotations

import datetime as _dt
import enum
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

from ..data.random_effect import FixedEffectDataConfiguration, RandomEffectDataConfiguration
from ..io.data_reader import FeatureShardConfiguration
from ..optimization.config import (GLMOptimizationConfiguration, OptimizerConfig, OptimizerType, RegularizationContext,
                                   RegularizationType)
from ..projector.projectors import INDEX_MAP

SECONDARY = "|"


class ModelOutputMode(str, enum.Enum):
    NONE = "NONE"
    BEST = "BEST"
    EXPLICIT = "EXPLICIT"
    TUNED = "TUNED"
    ALL = "ALL"


class HyperparameterTuningMode(str, enum.Enum):
    NONE = "NONE"
    RANDOM = "RANDOM"
    BAYESIAN = "BAYESIAN"


def parse_kv(s: str) -> Dict[str, str]:
    out = {}
    for part in s.split(","):
        part = part.strip()
        if not part:
            continue
        if "=" not in part:
            raise ValueError(f"expected key=value, got {part!r} in {s!r}")
        k, v = part.split("=", 1)
        out[k.strip()] = v.strip()
    return out


def parse_bool(s) -> bool:
    if isinstance(s, bool):
        return s
    v = str(s).strip().lower()
    if v in ("true", "1", "yes", "y"):
        return True
    if v in ("false", "0", "no", "n"):
        return False
    raise ValueError(f"not a boolean: {s}")


def parse_feature_shard_configuration(s: str) -> Dict[str, FeatureShardConfiguration]:
    kv = parse_kv(s)
    for req in ("name", "feature.bags"):
        if req not in kv:
            raise ValueError(f"feature shard configuration requires '{req}': {s}")
    bags = [b for b in kv["feature.bags"].split(SECONDARY) if b]
    return {kv["name"]: FeatureShardConfiguration(bags, parse_bool(kv.get("intercept", "true")))}


@dataclass
class CoordinateConfiguration:
    data_configuration: object
    optimization_configuration: GLMOptimizationConfiguration
    regularization_weights: List[float] = field(default_factory=list)

    @property
    def is_random_effect(self) -> bool:
        return isinstance(self.data_configuration, RandomEffectDataConfiguration)

    def expand_optimization_configurations(self) -> List[GLMOptimizationConfiguration]:
        """One config per λ, descending (CoordinateConfiguration.scala:71-78); NONE regularisation -> [0]."""
        oc = self.optimization_configuration
        if oc.regularization_context.regularization_type == RegularizationType.NONE or not self.regularization_weights:
            return [oc.with_reg_weight(oc.regularization_weight)]
        return [oc.with_reg_weight(w) for w in sorted(set(self.regularization_weights), reverse=True)]


def parse_coordinate_configuration(s: str) -> Dict[str, CoordinateConfiguration]:
    kv = parse_kv(s)
    for req in ("name", "feature.shard", "optimizer", "max.iter", "tolerance"):
        if req not in kv:
            raise ValueError(f"coordinate configuration requires '{req}': {s}")
    name = kv["name"]
    shard = kv["feature.shard"]
    min_parts = int(kv.get("min.partitions", "1"))
    oc = OptimizerConfig(OptimizerType.parse(kv["optimizer"]), int(kv["max.iter"]), float(kv["tolerance"]))
    reg = RegularizationType.parse(kv.get("regularization", "NONE"))
    if reg == RegularizationType.ELASTIC_NET:
        rc = RegularizationContext(reg, float(kv["reg.alpha"]) if "reg.alpha" in kv else None)
    else:
        rc = RegularizationContext(reg)
    weights = [float(x) for x in kv["reg.weights"].split(SECONDARY)] if "reg.weights" in kv else []
    if "random.effect.type" in kv:
        dc = RandomEffectDataConfiguration(
            kv["random.effect.type"], shard, min_parts,
            int(kv["active.data.bound"]) if "active.data.bound" in kv else None,
            int(kv["passive.data.bound"]) if "passive.data.bound" in kv else None,
            float(kv["features.to.samples.ratio"]) if "features.to.samples.ratio" in kv else None,
            INDEX_MAP)
        opt = GLMOptimizationConfiguration(oc, rc, 0.0)
    else:
        dc = FixedEffectDataConfiguration(shard, min_parts)
        opt = GLMOptimizationConfiguration(oc, rc, 0.0, float(kv.get("down.sampling.rate", "1.0")))
    return {name: CoordinateConfiguration(dc, opt, weights)}


def coordinate_configuration_to_string(name: str, cc: CoordinateConfiguration) -> str:
    dc, oc = cc.data_configuration, cc.optimization_configuration
    parts = [f"name={name}", f"feature.shard={dc.feature_shard_id}", f"min.partitions={dc.min_partitions}",
             f"optimizer={oc.optimizer_config.optimizer_type.value}",
             f"max.iter={oc.optimizer_config.maximum_iterations}", f"tolerance={oc.optimizer_config.tolerance}",
             f"regularization={oc.regularization_context.regularization_type.value}"]
    if oc.regularization_context.elastic_net_param is not None:
        parts.append(f"reg.alpha={oc.regularization_context.elastic_net_param}")
    if cc.regularization_weights:
        parts.append("reg.weights=" + SECONDARY.join(str(w) for w in cc.regularization_weights))
    if cc.is_random_effect:
        parts.append(f"random.effect.type={dc.random_effect_type}")
        if dc.active_data_upper_bound is not None:
            parts.append(f"active.data.bound={dc.active_data_upper_bound}")
        if dc.passive_data_lower_bound is not None:
            parts.append(f"passive.data.bound={dc.passive_data_lower_bound}")
        if dc.features_to_samples_ratio is not None:
            parts.append(f"features.to.samples.ratio={dc.features_to_samples_ratio}")
    elif oc.down_sampling_rate != 1.0:
        parts.append(f"down.sampling.rate={oc.down_sampling_rate}")
    return ",".join(parts)


def expand_game_configurations(coords: Dict[str, CoordinateConfiguration]) -> List[Dict[str, GLMOptimizationConfiguration]]:
    """Cartesian product of per-coordinate λ lists (GameTrainingDriver.prepareGameOptConfigs)."""
    configs: List[Dict[str, GLMOptimizationConfiguration]] = [{}]
    for cid, cc in coords.items():
        configs = [{**c, cid: oc} for c in configs for oc in cc.expand_optimization_configurations()]
    return configs


# ---------------------------------------------------------------- dates
def parse_date_range(s: str):
    a, b = s.split("-")
    d0 = _dt.datetime.strptime(a, "%Y%m%d").date()
    d1 = _dt.datetime.strptime(b, "%Y%m%d").date()
    if d1 < d0:
        raise ValueError(f"Invalid date range {s}")
    return d0, d1


def parse_days_range(s: str, today: Optional[_dt.date] = None):
    a, b = (int(x) for x in s.split("-"))
    today = today or _dt.date.today()
    if a < b:
        raise ValueError("days range must be 'start-end' with start >= end (days ago)")
    return today - _dt.timedelta(days=a), today - _dt.timedelta(days=b)


def expand_daily_dirs(base_dirs: Sequence[str], start: _dt.date, end: _dt.date) -> List[str]:
    out = []
    d = start
    while d <= end:
        for b in base_dirs:
            p = os.path.join(b, f"{d.year:04d}", f"{d.month:02d}", f"{d.day:02d}")
            if os.path.exists(p):
                out.append(p)
        d += _dt.timedelta(days=1)
    return out


def split_list(values: Optional[Sequence[str]]) -> List[str]:
    out = []
    for v in values or []:
        out.extend(x.strip() for x in str(v).split(",") if x.strip())
    return out


# --------------------------------------------------------------------------------------------------------------
# Config files: every driver flag can also come from a JSON / YAML mapping {flag-name: value}, and the parsed
# command line can be written back out (the round-trip the reference's ScoptParameter printer gives,
# ``CLI/io/scopt/ScoptParameter.scala:58-90``, as a file instead of a log line).

CONFIG_FILE_FLAG = "--config-file"
WRITE_CONFIG_FLAG = "--write-config"


def _long_option(action) -> Optional[str]:
    longs = [s for s in action.option_strings if s.startswith("--")]
    return longs[0] if longs else None


def _is_append(action) -> bool:
    import argparse
    return isinstance(action, argparse._AppendAction)


def load_config_file(path: str) -> Dict[str, object]:
    """A ``{flag-name: value}`` mapping from ``.json`` or ``.yaml``/``.yml`` (safe loader only)."""
    with open(path) as f:
        if path.endswith((".yaml", ".yml")):
            import yaml
            cfg = yaml.safe_load(f) or {}
        else:
            import json
            cfg = json.load(f)
    if not isinstance(cfg, dict):
        raise ValueError(f"{path}: a config file must hold a mapping of flag names to values")
    return cfg


def _scalar(v) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    return str(v)


def config_to_argv(parser, cfg: Dict[str, object]) -> List[str]:
    """Command-line tokens for a config mapping; keys are flag names with or without the leading ``--``."""
    known = {}
    for a in parser._actions:
        for s in a.option_strings:
            known[s] = a
    argv: List[str] = []
    for key, value in cfg.items():
        flag = key if key.startswith("--") else "--" + key.replace("_", "-")
        action = known.get(flag)
        if action is None:
            raise ValueError(f"unknown option {flag!r} in config file")
        if value is None:
            continue
        values = value if isinstance(value, (list, tuple)) else [value]
        if not _is_append(action) and isinstance(value, (list, tuple)):
            raise ValueError(f"option {flag!r} takes one value, got a list")
        for v in values:
            argv += [flag, _scalar(v)]
    return argv


def args_to_config(parser, args) -> Dict[str, object]:
    """The parsed options as a ``{flag-name: value}`` mapping that :func:`config_to_argv` turns back into ``args``."""
    out: Dict[str, object] = {}
    for a in parser._actions:
        flag = _long_option(a)
        if flag is None or flag in (CONFIG_FILE_FLAG, WRITE_CONFIG_FLAG) or not hasattr(args, a.dest):
            continue
        v = getattr(args, a.dest)
        if v is None or v == a.default:
            continue
        if isinstance(v, enum.Enum):
            v = v.value
        out[flag[2:]] = list(v) if isinstance(v, (list, tuple)) else v
    return out


def parse_args_with_config(parser, argv: Optional[Sequence[str]] = None):
    """``parser.parse_args`` that also accepts ``--config-file PATH`` (values from the file; a flag given on the
    command line replaces the file's value, for repeatable flags the whole list) and ``--write-config PATH`` (writes
    the effective options as JSON or YAML by extension)."""
    import sys
    argv = list(sys.argv[1:] if argv is None else argv)
    pre = _preparser()
    known, rest = pre.parse_known_args(argv)
    file_argv: List[str] = []
    if known.config_file:
        cfg = load_config_file(known.config_file)
        on_cli = {tok.split("=", 1)[0] for tok in rest if tok.startswith("--")}
        aliases = {}
        for a in parser._actions:
            for s in a.option_strings:
                aliases[s] = set(a.option_strings)
        cfg = {k: v for k, v in cfg.items()
               if not (aliases.get(k if k.startswith("--") else "--" + k.replace("_", "-"), set()) & on_cli)}
        file_argv = config_to_argv(parser, cfg)
    args = parser.parse_args(file_argv + rest)
    if known.write_config:
        write_config_file(known.write_config, args_to_config(parser, args))
    return args


def write_config_file(path: str, cfg: Dict[str, object]) -> None:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w") as f:
        if path.endswith((".yaml", ".yml")):
            import yaml
            yaml.safe_dump(cfg, f, sort_keys=True, default_flow_style=False)
        else:
            import json
            json.dump(cfg, f, indent=2, sort_keys=True)


def _preparser():
    import argparse
    pre = argparse.ArgumentParser(add_help=False, allow_abbrev=False)
    pre.add_argument(CONFIG_FILE_FLAG)
    pre.add_argument(WRITE_CONFIG_FLAG)
    return pre


def add_config_arguments(p) -> None:
    """Registers the config-file flags on a driver parser (so ``--help`` lists them)."""
    p.add_argument(CONFIG_FILE_FLAG, help="JSON/YAML mapping of flag names to values; command-line flags win")
    p.add_argument(WRITE_CONFIG_FLAG, help="write the effective options to this JSON/YAML file")
