"""Process-group plumbing and the data-parallel GLM wrapper (Spark treeAggregate -> RCCL all-reduce).

One process per GPU (``torch.distributed`` backend ``nccl`` == RCCL over xGMI on ROCm; ``gloo`` on CPU for
tests, the analogue of the reference's Spark ``local[*]``). Every rank owns a ROW SHARD of the data and a
REPLICA of the optimizer state; each function evaluation all-reduces ONE packed fp64 buffer ``[G | F | S]``
(``ValueAndGradientAggregator.scala:243-247`` treeAggregate of (F, S, G)). Because every
rank then applies the identical deterministic optimizer update, coefficients are never broadcast (C5 removed).

Message sizing for xGMI: D = 1M fp64 = 8 MB per evaluation; a ring all-reduce moves 2(P-1)/P x 8 MB per rank
(~14 MB at P = 8), i.e. ~0.1 ms on one 153 GB/s link against a ~40 ms evaluation pass. That is small, but not
free at the END of a pass: :class:`DistributedGLMData` therefore buckets the gradient by column-tile ranges of
equal transpose work and all-reduces each bucket while the transpose kernels of the later buckets still run
(RCCL's stream waits on the compute stream per bucket), so only the last bucket's collective is exposed.

The reference's ``treeAggregateDepth`` knob (``GameEstimator.scala:111-114, 587-592``) maps to the RCCL
all-reduce algorithm (:func:`set_allreduce_algo`: ring / tree / RCCL's own choice).
"""
from __future__ import annotations

import datetime
import os
from typing import Optional

import torch
import torch.distributed as dist

from ..utils.timing import trace_range


def env_world() -> tuple[int, int, int]:
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def force_collectives() -> bool:
    """``PML_FORCE_DIST=1``: a world of ONE rank still initialises the process group and routes every aggregate
    through the collectives (RCCL on a single GPU: the multi-rank code path — bucketed async all-reduce, device
    all-to-all, all-gather / reduce-scatter — executed on hardware with the trivial group)."""
    return os.environ.get("PML_FORCE_DIST", "0") == "1"


def init_distributed(backend: Optional[str] = None, timeout_s: int = 1800) -> tuple[int, int, int]:
    """Initialise the default process group from torchrun env vars (no-op for world size 1 unless
    ``PML_FORCE_DIST=1``)."""
    rank, world, local = env_world()
    from ..utils.watchdog import start_watchdog
    start_watchdog()  # PML_WATCHDOG_S: abort this rank (-> torchrun aborts the group) when progress stops
    if (world > 1 or force_collectives()) and not dist.is_initialized():
        # a collective that exceeds ``timeout_s`` raises instead of hanging (RCCL async error handling)
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        timeout_s = int(os.environ.get("PML_COLLECTIVE_TIMEOUT_S", timeout_s))
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        if backend is None:
            backend = os.environ.get("PML_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local % torch.cuda.device_count())
        dist.init_process_group(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
    return rank, world, local


ALLREDUCE_ALGOS = ("auto", "ring", "tree")
_EXPLICIT_ALGO: Optional[str] = None


def set_allreduce_algo(algo: Optional[str] = None, tree_depth: Optional[int] = None) -> str:
    """Choose the RCCL all-reduce algorithm — the analogue of the reference's ``treeAggregateDepth``
    (``photon-api/.../estimators/GameEstimator.scala:111-114``; auto depth 2 for D >= 200k at ``:587-592``):
    ``ring`` / ``tree`` set ``NCCL_ALGO`` (which RCCL reads when it creates a communicator; torch creates them
    lazily at the first collective, so call this before any collective runs), ``auto`` leaves RCCL's tuner in
    charge. Without an explicit ``algo``, a tree-aggregate depth >= 2 selects ``tree`` (a hierarchical reduction,
    like a deeper treeAggregate) and depth 1 ``auto``. A ``NCCL_ALGO`` already set in the environment wins.
    An explicit ``algo`` (e.g. ``--allreduce-algo``) sticks: later depth-only calls do not change it. Returns
    the effective choice."""
    global _EXPLICIT_ALGO
    if algo is None:
        if _EXPLICIT_ALGO is not None:
            return _EXPLICIT_ALGO
        algo = "tree" if (tree_depth or 1) >= 2 else "auto"
    else:
        _EXPLICIT_ALGO = algo.lower()
    algo = algo.lower()
    if algo not in ALLREDUCE_ALGOS:
        raise ValueError(f"unknown all-reduce algorithm {algo!r}, expected one of {ALLREDUCE_ALGOS}")
    if "NCCL_ALGO" in os.environ and os.environ.get("PML_NCCL_ALGO_SET") != "1":
        return os.environ["NCCL_ALGO"].lower()
    if algo == "auto":
        if os.environ.get("PML_NCCL_ALGO_SET") == "1":
            os.environ.pop("NCCL_ALGO", None)
            os.environ.pop("PML_NCCL_ALGO_SET", None)
        return "auto"
    os.environ["NCCL_ALGO"] = {"ring": "Ring", "tree": "Tree"}[algo]
    os.environ["PML_NCCL_ALGO_SET"] = "1"       # ours, may be changed again
    return algo


def is_dist() -> bool:
    return (dist.is_available() and dist.is_initialized()
            and (dist.get_world_size() > 1 or force_collectives()))


def world_size() -> int:
    return dist.get_world_size() if is_dist() else 1


def rank() -> int:
    return dist.get_rank() if is_dist() else 0


def all_reduce_(t: torch.Tensor, op=None, group=None) -> torch.Tensor:
    if is_dist():
        dist.all_reduce(t, op=op or dist.ReduceOp.SUM, group=group)
    return t


def all_reduce_scalar(x: float, op: str = "sum", device=None, group=None) -> float:
    if not is_dist():
        return float(x)
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    ops = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}
    dist.all_reduce(t, op=ops[op], group=group)
    return float(t.item())


def barrier(group=None):
    if is_dist():
        dist.barrier(group=group)


def device_identity(device) -> str:
    """A string naming the PHYSICAL device a rank computes on: host + PCI domain/bus/device + UUID for a GPU,
    host + "cpu" otherwise. Two ranks sharing one GPU (rehearsal runs) get the same identity."""
    import socket
    host = socket.gethostname()
    d = torch.device(device)
    if d.type != "cuda":
        return f"{host}:cpu"
    idx = d.index if d.index is not None else torch.cuda.current_device()
    p = torch.cuda.get_device_properties(idx)
    pci = f"{getattr(p, 'pci_domain_id', 0):04x}:{getattr(p, 'pci_bus_id', 0):02x}:{getattr(p, 'pci_device_id', 0):02x}"
    return f"{host}:{pci}:{getattr(p, 'uuid', '')}"


def distinct_devices(device) -> int:
    """Number of distinct physical devices over all ranks (all-gather of :func:`device_identity`). Benchmarks
    report THIS as ``n_gpus`` (the rank count goes in ``n_ranks``)."""
    ident = device_identity(device)
    if not is_dist():
        return 1
    out = [None] * world_size()
    dist.all_gather_object(out, ident)
    return len(set(out))


def check_finite_(t: torch.Tensor, what: str):
    """NaN/Inf guard on an all-reduced buffer (SURVEY §5 failure detection)."""
    if not bool(torch.isfinite(t).all()):
        raise FloatingPointError(f"non-finite values in all-reduced {what}")


def read_tail_checked(buf: torch.Tensor, start: int, what: str, guard: bool = True) -> list:
    """``buf[start:]`` as host floats, with the NaN/Inf guard of the WHOLE buffer riding on the same readback: the
    finiteness flag is reduced on the device and appended to the tail, so guarding costs no extra host
    synchronisation per collective (the [F, S] scalars are read anyway)."""
    tail = buf[start:]
    if not guard:
        return tail.tolist()
    vals = torch.cat([tail, torch.isfinite(buf).all().to(buf.dtype).reshape(1)]).tolist()
    if vals[-1] != 1.0:
        raise FloatingPointError(f"non-finite values in all-reduced {what}")
    return vals[:-1]


class DistributedGLMData:
    """Wraps a local row shard; every aggregate is summed over the process group with one collective."""

    def __init__(self, local, group=None, nan_guard: bool = True):
        self.local = local
        self.group = group
        self.nan_guard = nan_guard
        self.dim = local.dim
        self.device = local.device
        n = torch.tensor([float(local.n_rows)], dtype=torch.float64, device=self._comm_device())
        all_reduce_(n, group=group)
        self.n_rows = int(n.item())
        self.local_rows = local.n_rows
        # Overlapped C1: gradient buckets reduced while the transpose pass still runs (needs the bucketed device
        # path and ONE feature order on every rank — the reduction happens in the device's permuted order).
        self.buckets = int(os.environ.get("PML_GRAD_BUCKETS", "4"))
        self.overlap = False
        if is_dist() and self.buckets > 1 and hasattr(local, "value_grad_packed_overlap"):
            fp = local.perm_fingerprint()
            lo = all_reduce_scalar(fp, "min", group=group)
            hi = all_reduce_scalar(fp, "max", group=group)
            self.overlap = lo == hi and local.grad_buckets(self.buckets) is not None

    def _comm_device(self):
        if is_dist() and dist.get_backend(self.group) == "nccl":
            return self.local.device
        return torch.device("cpu")

    @property
    def track_hessian(self):
        return getattr(self.local, "track_hessian", False)

    @track_hessian.setter
    def track_hessian(self, v):
        if hasattr(self.local, "track_hessian"):
            self.local.track_hessian = v

    def _packed_overlap(self, fn, *args) -> torch.Tensor:
        """Bucketed pass: each final gradient slice (and [F, S]) is all-reduced asynchronously while the
        transpose kernels of the next buckets run; RCCL's stream waits on the compute stream at each call, so
        ordering is by construction. Same bits as the one-shot path (tiles are independent)."""
        works = []

        def start(t):
            works.append(dist.all_reduce(t, group=self.group, async_op=True))

        with trace_range(f"C1 overlapped all-reduce {fn} [{self.dim + 2} fp64, {self.buckets} buckets]"):
            buf = getattr(self.local, fn + "_packed_overlap")(*args, start, nb=self.buckets)
            for w in works:
                w.wait()
        if self.local.old_of_new is not None:
            buf[: self.dim] = self.local._unperm(buf[: self.dim].clone())
        return buf

    def _packed(self, fn, *args) -> torch.Tensor:
        local = self.local
        if self.overlap and fn in ("value_grad", "hv"):
            return self._packed_overlap(fn, *args)
        if hasattr(local, fn + "_packed"):
            buf = getattr(local, fn + "_packed")(*args)
        else:
            a, b, *rest = getattr(local, fn + "_sums")(*args)
            if fn == "value_grad":
                f, s, g = a, b, rest[0]
                buf = torch.cat([g.to(torch.float64), torch.tensor([f, s], dtype=torch.float64, device=g.device)])
            else:
                h, p = a, b
                buf = torch.cat([h.to(torch.float64), torch.tensor([0.0, p], dtype=torch.float64, device=h.device)])
        dev = self._comm_device()
        with trace_range(f"C1 all-reduce {fn} [{buf.numel()} fp64]"):
            if buf.device != dev:
                tmp = buf.to(dev)
                all_reduce_(tmp, group=self.group)
                buf = tmp.to(buf.device)
            else:
                all_reduce_(buf, group=self.group)
        return buf      # the NaN guard rides on the caller's scalar readback (read_tail_checked)

    # margin-space line search: trials need two scalars per rank; the accepted step one (overlapped) reduction
    def ls_begin(self, w0_eff, shift0, d_eff, d_shift, t0: float = 1.0, loss=None) -> bool:
        ok = bool(getattr(self.local, "ls_begin", lambda *a, **k: False)(w0_eff, shift0, d_eff, d_shift, t0, loss))
        return all_reduce_scalar(1.0 if ok else 0.0, "min", device=self._scalar_device(), group=self.group) > 0

    def step_begin(self, w_eff, shift) -> bool:
        """TRON margin-space trial (DeviceGLMData.step_begin) on every rank, or on none."""
        ok = bool(getattr(self.local, "step_begin", lambda *a: False)(w_eff, shift))
        return all_reduce_scalar(1.0 if ok else 0.0, "min", device=self._scalar_device(), group=self.group) > 0

    def step_add(self, alpha: float):
        self.local.step_add(alpha)

    def _scalar_device(self):
        return self.local.device if dist.get_backend(self.group) == "nccl" else None

    def ls_eval(self, loss, t: float):
        f, d = self.local.ls_eval(loss, t)
        dev = self._comm_device()
        v = torch.tensor([f, d], dtype=torch.float64, device=dev)
        all_reduce_(v, group=self.group)
        f, d = read_tail_checked(v, 0, "line search", self.nan_guard)
        return f, d

    def zero_point_sums(self, loss, margin_shift):
        """[F, S, ||c||^2, ||X||_F^2] summed over the ranks (one 4-scalar all-reduce): by Cauchy-Schwarz
        ||sum_r X_r^T c_r|| <= sqrt(sum ||X_r||_F^2) sqrt(sum ||c_r||^2), so the bound stays valid."""
        if not hasattr(self.local, "zero_point_sums"):
            raise AttributeError("zero_point_sums")
        t = torch.tensor(self.local.zero_point_sums(loss, margin_shift), dtype=torch.float64,
                         device=self._comm_device())
        all_reduce_(t, group=self.group)
        return t.tolist()

    def ls_finish_sums(self, loss, t: float, w_eff, shift, need_s: bool = True):
        if self.overlap and hasattr(self.local, "ls_finish_packed"):
            works = []

            def start(x):
                works.append(dist.all_reduce(x, group=self.group, async_op=True))

            with trace_range(f"C1 overlapped all-reduce (accepted step) [{self.dim + 2} fp64]"):
                buf = self.local.ls_finish_packed(loss, t, w_eff, shift, need_s, start_reduce=start, nb=self.buckets)
                for w in works:
                    w.wait()
            if self.local.old_of_new is not None:
                buf[: self.dim] = self.local._unperm(buf[: self.dim].clone())
        else:
            f, s_, g = self.local.ls_finish_sums(loss, t, w_eff, shift, need_s)
            buf = torch.cat([g.to(torch.float64), torch.tensor([f, s_], dtype=torch.float64, device=g.device)])
            dev = self._comm_device()
            tmp = buf.to(dev)
            all_reduce_(tmp, group=self.group)
            buf = tmp.to(buf.device)
        fs = read_tail_checked(buf, self.dim, "ls_finish", self.nan_guard)
        return fs[0], fs[1], buf[: self.dim]

    def value_grad_sums(self, loss, w_eff, margin_shift):
        buf = self._packed("value_grad", loss, w_eff, margin_shift)
        fs = read_tail_checked(buf, self.dim, "value_grad", self.nan_guard)
        return fs[0], fs[1], buf[: self.dim]

    def hv_sums(self, loss, w_eff, margin_shift, v_eff, v_shift):
        buf = self._packed("hv", loss, w_eff, margin_shift, v_eff, v_shift)
        fs = read_tail_checked(buf, self.dim, "hv", self.nan_guard)
        return buf[: self.dim], fs[1]

    def hdiag_sums(self, loss, w):
        d = self.local.hdiag_sums(loss, w).to(torch.float64)
        dev = self._comm_device()
        t = d.to(dev)
        all_reduce_(t, group=self.group)
        return t.to(d.device)

    def margins(self, w, margin_shift=0.0, with_offsets=False):
        return self.local.margins(w, margin_shift, with_offsets)
