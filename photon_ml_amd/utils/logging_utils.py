"""PhotonLogger equivalent and event emitter.

Reference: ``photon-lib/.../util/PhotonLogger.scala:34-553`` (a logger that writes a local file under the output
directory and echoes to stdout; levels set per driver), ``photon-client/.../event/{Event,EventEmitter,
EventListener}.scala`` (setup / training start / training finish / optimisation-log events delivered to
listeners registered by class name).
"""
from __future__ import annotations

import importlib
import json
import logging
import os
import sys
import time
from dataclasses import asdict, dataclass, field
from typing import Any, Callable, Dict, List, Optional

LEVELS = {"TRACE": 5, "DEBUG": logging.DEBUG, "INFO": logging.INFO, "WARN": logging.WARNING,
          "WARNING": logging.WARNING, "ERROR": logging.ERROR}


class PhotonLogger:
    """File + stdout logger rooted at ``log_dir``; ``close()`` flushes (the reference copies to HDFS)."""

    def __init__(self, log_dir: str, level: str = "INFO", name: str = "photon_ml_amd", rank: int = 0):
        os.makedirs(log_dir, exist_ok=True)
        self.path = os.path.join(log_dir, "log-message.txt" if rank == 0 else f"log-message-rank{rank}.txt")
        self.logger = logging.getLogger(name)
        self.logger.setLevel(LEVELS.get(str(level).upper(), logging.INFO))
        self.logger.propagate = False
        for h in list(self.logger.handlers):
            self.logger.removeHandler(h)
        fmt = logging.Formatter("%(asctime)s %(levelname)s %(name)s: %(message)s")
        self.fh = logging.FileHandler(self.path)
        self.fh.setFormatter(fmt)
        self.logger.addHandler(self.fh)
        if rank == 0:
            sh = logging.StreamHandler(sys.stdout)
            sh.setFormatter(fmt)
            self.logger.addHandler(sh)

    def __getattr__(self, item):
        return getattr(self.logger, item)

    def close(self):
        self.fh.flush()
        self.fh.close()
        self.logger.removeHandler(self.fh)


# ----------------------------------------------------------------------------------------------------------------
@dataclass
class Event:
    name: str
    time: float = field(default_factory=time.time)
    payload: Dict[str, Any] = field(default_factory=dict)


class EventListener:
    def handle(self, event: Event):  # pragma: no cover - interface
        raise NotImplementedError

    def close(self):
        pass


class JsonLinesEventListener(EventListener):
    """Appends every event as one JSON line (per-iteration timelines for observability)."""

    def __init__(self, path: str):
        os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
        self.f = open(path, "a")

    def handle(self, event):
        self.f.write(json.dumps({"event": event.name, "time": event.time, **event.payload}, default=str) + "\n")
        self.f.flush()

    def close(self):
        self.f.close()


class EventEmitter:
    def __init__(self):
        self.listeners: List[EventListener] = []

    def register(self, listener: EventListener):
        self.listeners.append(listener)

    def register_by_name(self, class_path: str, *args):
        mod, cls = class_path.rsplit(".", 1)
        self.register(getattr(importlib.import_module(mod), cls)(*args))

    def emit(self, name: str, **payload):
        ev = Event(name, payload=payload)
        for l in self.listeners:
            l.handle(ev)

    def close(self):
        for l in self.listeners:
            l.close()
