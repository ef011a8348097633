"""Rank-failure / hang watchdog (SURVEY §5 "failure detection": RCCL timeout -> abort all).

The reference leaves failure handling to Spark (task retry + lineage recomputation). With one process per GPU
and blocking RCCL collectives, the failure mode to guard against is a HANG: a peer rank died or diverged, and
the survivors wait in an all-reduce forever. Three layers:

1. ``init_distributed`` sets a finite collective timeout and RCCL async error handling
   (``TORCH_NCCL_ASYNC_ERROR_HANDLING=1``): a collective that times out raises / tears the communicator down.
2. :class:`Watchdog` — a daemon thread fed by heartbeats (every ``Timed`` block and ``trace_range`` exit beats:
   optimizer iterations, evaluation passes, collectives, coordinate updates). If no heartbeat arrives for
   ``timeout_s`` it dumps every thread's Python stack (``faulthandler``) and hard-exits the process with
   ``EXIT_CODE``; ``torch.distributed.run`` then sees a failed worker and terminates the whole group, i.e. one
   stuck rank aborts the job instead of holding 8 GPUs idle.
3. NaN/Inf guards on every all-reduced buffer (``parallel.dist.check_finite_``) and checkpoint/resume
   (``utils.checkpoint``) so an aborted job restarts from the last coordinate-descent iteration.

Enabled by drivers/benches with ``PML_WATCHDOG_S=<seconds>`` (or explicitly via :func:`start_watchdog`).
"""
from __future__ import annotations

import faulthandler
import logging
import os
import sys
import threading
import time
from typing import Optional

EXIT_CODE = 75
log = logging.getLogger("photon_ml_amd.watchdog")

_last_beat = time.monotonic()
_active: Optional["Watchdog"] = None


def heartbeat():
    """Record progress (cheap: one monotonic clock read)."""
    global _last_beat
    _last_beat = time.monotonic()


class Watchdog:
    def __init__(self, timeout_s: float, poll_s: Optional[float] = None, exit_code: int = EXIT_CODE):
        self.timeout_s = float(timeout_s)
        self.poll_s = poll_s if poll_s is not None else max(0.05, min(10.0, self.timeout_s / 10))
        self.exit_code = exit_code
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, name="pml-watchdog", daemon=True)

    def start(self) -> "Watchdog":
        heartbeat()
        self._thread.start()
        return self

    def stop(self):
        self._stop.set()

    def _run(self):
        while not self._stop.wait(self.poll_s):
            idle = time.monotonic() - _last_beat
            if idle > self.timeout_s:
                rank = os.environ.get("RANK", "0")
                msg = (f"[photon_ml_amd watchdog] rank {rank}: no progress for {idle:.1f} s (limit {self.timeout_s} s)"
                       f" -- a peer rank probably failed or a collective is stuck; aborting with exit code "
                       f"{self.exit_code}")
                print(msg, file=sys.stderr, flush=True)
                log.error(msg)
                faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
                sys.stderr.flush()
                os._exit(self.exit_code)


def start_watchdog(timeout_s: Optional[float] = None) -> Optional[Watchdog]:
    """Start the process-wide watchdog (``timeout_s`` or ``$PML_WATCHDOG_S``; no-op when neither is set)."""
    global _active
    if timeout_s is None:
        env = os.environ.get("PML_WATCHDOG_S")
        if not env:
            return None
        timeout_s = float(env)
    if _active is not None:
        _active.stop()
    _active = Watchdog(timeout_s).start()
    return _active


def stop_watchdog():
    global _active
    if _active is not None:
        _active.stop()
        _active = None
