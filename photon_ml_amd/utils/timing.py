"""``Timed`` blocks (``photon-lib/.../util/Timed.scala:33-77``) plus tracing for the profiler.

* ``Timed(msg)`` logs the wall time of a named block and appends it to the in-process ``TIMELINE`` (drivers dump
  it as JSON: ``dump_timeline``).
* With ``PML_TRACE=1`` every ``Timed`` block and every ``trace_range`` is also a roctx range (``torch.cuda.nvtx``
  maps to roctx on ROCm), so ``rocprofv3 --marker-trace`` shows optimizer iterations / evaluation passes /
  coordinate updates around the kernel timeline (SURVEY §5 tracing: "roctx ranges on every K#/C# launch").
* ``PML_TIMELINE=<path>`` appends one JSON line per closed block (name, start, seconds, rank) for per-iteration
  timelines of eval / comm / optimizer phases.
"""
from __future__ import annotations

import json
import logging
import os
import time
from collections import defaultdict
from contextlib import contextmanager

from .watchdog import heartbeat

TIMELINE = defaultdict(list)
_TRACE = os.environ.get("PML_TRACE", "0") == "1"
_TIMELINE_PATH = os.environ.get("PML_TIMELINE")
# PML_SYNC_TIMED=1: every Timed block synchronises the device on entry and exit, so its wall time is the device-
# complete time of the work queued inside it (phase tables of the one-shot build / cold sweep; never in a timed run)
_SYNC = os.environ.get("PML_SYNC_TIMED", "0") == "1"


def _device_sync():
    if _SYNC:
        import torch
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()


def _roctx_push(name: str):
    if _TRACE:
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.nvtx.range_push(name)
                return True
        except Exception:  # pragma: no cover
            pass
    return False


def _roctx_pop():
    import torch
    torch.cuda.nvtx.range_pop()


def _emit(name: str, t0: float, dt: float):
    TIMELINE[name].append(dt)
    if _TIMELINE_PATH:
        try:
            rank = int(os.environ.get("RANK", "0"))
            with open(_TIMELINE_PATH, "a") as f:
                f.write(json.dumps({"name": name, "start": t0, "seconds": dt, "rank": rank}) + "\n")
        except OSError:  # pragma: no cover
            pass


class Timed:
    def __init__(self, msg: str, logger=None, level=logging.INFO):
        self.msg = msg
        self.logger = logger or logging.getLogger("photon_ml_amd")
        self.level = level

    def __enter__(self):
        _device_sync()
        self._pushed = _roctx_push(self.msg)
        self.wall0 = time.time()
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        _device_sync()
        heartbeat()
        self.elapsed = time.perf_counter() - self.t0
        if self._pushed:
            _roctx_pop()
        _emit(self.msg, self.wall0, self.elapsed)
        self.logger.log(self.level, "%s: %.3f s", self.msg, self.elapsed)
        return False


@contextmanager
def trace_range(name: str):
    """Lightweight roctx range (no logging) for hot paths: optimizer iterations, evaluation passes, collectives."""
    pushed = _roctx_push(name)
    try:
        yield
    finally:
        heartbeat()
        if pushed:
            _roctx_pop()


def phase(msg: str) -> Timed:
    """A DEBUG-level ``Timed`` block for build / setup phases (device-complete with ``PML_SYNC_TIMED=1``)."""
    return Timed(msg, logging.getLogger("photon_ml_amd.phase"), logging.DEBUG)


def timed(msg: str, fn, *args, logger=None, **kw):
    with Timed(msg, logger):
        return fn(*args, **kw)


def dump_timeline(path: str):
    """Write the aggregated per-block timings ({name: {count, total_s, mean_s}}) as JSON."""
    agg = {k: {"count": len(v), "total_s": float(sum(v)), "mean_s": float(sum(v) / len(v))}
           for k, v in TIMELINE.items() if v}
    with open(path, "w") as f:
        json.dump(agg, f, indent=2, sort_keys=True)
    return agg
