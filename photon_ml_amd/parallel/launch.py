"""Self-launch of the multi-GPU entry points (one process per GPU).

``python bench.py --gpus 8`` run WITHOUT a launcher must not quietly measure one rank: :func:`relaunch_if_needed`
starts ``torch.distributed.run`` with one rank per requested GPU as a CHILD process (before this process touches
the GPU — a process that initialised HIP must never exec another program) and returns the child's exit code,
which the caller exits with. Under a launcher (``WORLD_SIZE`` set) a world size different from ``--gpus`` is an
error, not a warning.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
from typing import List, Optional


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_command(n: int, script: str, argv: List[str], port: Optional[int] = None) -> List[str]:
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port or free_port()), script, *argv]


def relaunch_if_needed(gpus: int, script: str, argv: List[str]) -> Optional[int]:
    """None: carry on in this process (single GPU, or already one rank of a launched group of the right size).
    Otherwise the exit code of the launched group. Raises SystemExit(2) on a world-size mismatch."""
    world = os.environ.get("WORLD_SIZE")
    if world is not None:
        if int(world) != gpus:
            print(f"error: --gpus {gpus} but WORLD_SIZE={world}: refusing to report a {world}-rank run as "
                  f"{gpus} GPUs", file=sys.stderr, flush=True)
            raise SystemExit(2)
        return None
    if gpus <= 1:
        return None
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC for RCCL on this host driver
    cmd = launcher_command(gpus, os.path.abspath(script), argv)
    print(f"[launch] {gpus} GPUs requested without a launcher: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env)
