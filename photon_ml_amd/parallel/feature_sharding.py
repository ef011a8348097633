"""Feature (column) sharding of the GLM optimizer state — the GLM analogue of ZeRO / tensor parallelism.

SURVEY §2.10: the reference replicates the coefficients on every executor (``sc.broadcast`` per evaluation,
``DistributedObjectiveFunction.scala:57-58``) and keeps the whole Breeze L-BFGS state on the driver, which caps
the model at what one JVM holds. Here, for models too large to replicate (D ~ 1e8-1e9 coefficients: w, g and
the 2m-vector L-BFGS history are 8 B x D x (2m + 4) ~ 190 GB at D = 1e9, m = 10), every rank keeps ONE
contiguous feature slice of every optimizer vector, while the data stays row-sharded with all D columns:

    evaluation:  all-gather w (8·D bytes)  ->  local fused value+gradient pass over the row shard (HIP kernels)
                 ->  reduce-scatter G (the same bytes as the replicated all-reduce, split RS + AG)  +  one
                 2-scalar all-reduce of (F, S)
    optimizer:   every vector op runs on the D/P slice; every inner product is a local partial + all-reduce
                 (``optimization.vector_space.ShardedSpace``); the L-BFGS two-loop is the vector-free variant
                 (one batched Gram all-reduce per iteration, ``lbfgs._History._apply_inverse_gram``).
    line search: in MARGIN space like the replicated path (the local row shard caches its margins): one
                 all-gather of the direction + one forward pass, then 2 scalars all-reduced per trial; TRON trial
                 points likewise come from the tracked step margins (no forward pass).

Memory per rank for the optimizer drops from (2m + 4)·8·D to (2m + 4)·8·D/P + 16·D (the gathered w and the
full-length local gradient of one pass). Communication per evaluation is unchanged versus the replicated
all-reduce (reduce-scatter + all-gather == all-reduce on a ring), so the sharded path costs no extra xGMI bytes.
On RCCL the collectives are ``all_gather_into_tensor`` / ``reduce_scatter_tensor`` on padded equal chunks; gloo
(CPU tests) falls back to all-reduce + slice.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

from ..function.objective import GLMObjective
from ..normalization.context import NormalizationContext, no_normalization
from ..optimization.vector_space import ShardedSpace, active_space
from ..utils.timing import trace_range
from .dist import is_dist


@dataclass(frozen=True)
class FeatureShardLayout:
    """Contiguous, equal (padded) feature chunks: rank r owns [lo, hi) of the D coefficients."""

    dim: int
    world: int
    rank: int

    @property
    def chunk(self) -> int:
        return max(1, -(-self.dim // self.world))

    @property
    def lo(self) -> int:
        return min(self.dim, self.rank * self.chunk)

    @property
    def hi(self) -> int:
        return min(self.dim, self.lo + self.chunk)

    @property
    def size(self) -> int:
        return self.hi - self.lo

    def slice(self, full: torch.Tensor) -> torch.Tensor:
        return full[self.lo:self.hi]

    @staticmethod
    def current(dim: int, group=None) -> "FeatureShardLayout":
        if is_dist():
            return FeatureShardLayout(dim, dist.get_world_size(group), dist.get_rank(group))
        return FeatureShardLayout(dim, 1, 0)


def _nccl(group) -> bool:
    return is_dist() and dist.get_backend(group) == "nccl"


def all_gather_shards(shard: torch.Tensor, layout: FeatureShardLayout, group=None) -> torch.Tensor:
    """Full D-vector from every rank's slice."""
    if layout.world == 1:
        return shard
    c = layout.chunk
    buf = torch.zeros(c, dtype=shard.dtype, device=shard.device)
    buf[: shard.numel()] = shard
    with trace_range(f"C5' all-gather w [{layout.dim}]"):
        if _nccl(group):
            out = torch.empty(c * layout.world, dtype=shard.dtype, device=shard.device)
            dist.all_gather_into_tensor(out, buf, group=group)
        else:
            parts = [torch.empty(c, dtype=shard.dtype) for _ in range(layout.world)]
            dist.all_gather(parts, buf.cpu(), group=group)
            out = torch.cat(parts).to(shard.device)
    return out[: layout.dim]


def reduce_scatter_full(full: torch.Tensor, layout: FeatureShardLayout, group=None) -> torch.Tensor:
    """This rank's slice of the sum over ranks of a full D-vector."""
    if layout.world == 1:
        return full
    c = layout.chunk
    with trace_range(f"C1' reduce-scatter g [{layout.dim}]"):
        if _nccl(group):
            buf = torch.zeros(c * layout.world, dtype=full.dtype, device=full.device)
            buf[: layout.dim] = full
            out = torch.empty(c, dtype=full.dtype, device=full.device)
            dist.reduce_scatter_tensor(out, buf, group=group)
            return out[: layout.size]
        t = full.detach().cpu().clone()
        dist.all_reduce(t, group=group)
        return layout.slice(t).to(full.device)


def _all_reduce_small(vals, device, group=None):
    t = torch.tensor(vals, dtype=torch.float64)
    if is_dist():
        t = t.to(device) if _nccl(group) else t
        dist.all_reduce(t, group=group)
    return t.cpu().tolist()


class FeatureShardedObjective:
    """:class:`GLMObjective` with sharded coefficient / gradient / Hessian-vector vectors.

    ``data`` is the LOCAL row shard (any GLM data backend: HIP ``DeviceGLMData`` or the torch reference) with
    every feature column; the normalization context holds full-length factors/shifts (sliced here).
    """

    def __init__(self, objective: GLMObjective, layout: FeatureShardLayout, group=None):
        self.obj = objective
        self.layout = layout
        self.group = group
        self.n_value_grad = 0
        self.n_hv = 0

    @property
    def loss(self):
        return self.obj.loss

    @property
    def l2_weight(self) -> float:
        return self.obj.l2_weight

    @property
    def twice_differentiable(self) -> bool:
        return self.obj.twice_differentiable

    def _norm_slice(self, v: Optional[torch.Tensor], like: torch.Tensor):
        return None if v is None else self.layout.slice(v).to(like)

    def _finalize(self, g_shard: torch.Tensor, prefactor: float) -> torch.Tensor:
        norm = self.obj.normalization
        out = g_shard
        sh = self._norm_slice(norm.shifts, out)
        if sh is not None:
            out = out - sh * prefactor
        fa = self._norm_slice(norm.factors, out)
        if fa is not None:
            out = out * fa
        return out

    def calculate(self, data, w_shard: torch.Tensor):
        self.n_value_grad += 1
        w = all_gather_shards(w_shard, self.layout, self.group)
        w_eff, shift = self.obj.normalization.effective(w)
        f, s, G = data.value_grad_sums(self.obj.loss, w_eff, shift)
        g_shard = reduce_scatter_full(G.to(torch.float64), self.layout, self.group)
        f, s = _all_reduce_small([f, s], G.device, self.group)
        grad = self._finalize(g_shard, s)
        if self.obj.l2_weight > 0:
            f += 0.5 * self.obj.l2_weight * float(torch.dot(w, w))  # w is whole here: no extra collective
            grad = grad + self.obj.l2_weight * w_shard
        return f, grad

    def value(self, data, w_shard):
        return self.calculate(data, w_shard)[0]

    def hessian_vector(self, data, w_shard: torch.Tensor, v_shard: torch.Tensor) -> torch.Tensor:
        if not self.twice_differentiable:
            raise NotImplementedError(f"{self.obj.loss} has no Hessian")
        self.n_hv += 1
        norm = self.obj.normalization
        w = all_gather_shards(w_shard, self.layout, self.group)
        v = all_gather_shards(v_shard, self.layout, self.group)
        w_eff, shift = norm.effective(w)
        v_eff = v * norm.factors.to(v) if norm.factors is not None else v
        v_shift = float(torch.dot(v_eff, norm.shifts.to(v_eff))) if norm.shifts is not None else 0.0
        h, p = data.hv_sums(self.obj.loss, w_eff, shift, v_eff, v_shift)
        h_shard = reduce_scatter_full(h.to(torch.float64), self.layout, self.group)
        p = _all_reduce_small([p], h.device, self.group)[0]
        hv = self._finalize(h_shard, p)
        if self.obj.l2_weight > 0:
            hv = hv + self.obj.l2_weight * v_shard
        return hv

    def hessian_diagonal(self, data, w_shard: torch.Tensor) -> torch.Tensor:
        w = all_gather_shards(w_shard, self.layout, self.group)
        d = reduce_scatter_full(data.hdiag_sums(self.obj.loss, w).to(torch.float64), self.layout, self.group)
        return d + self.obj.l2_weight if self.obj.l2_weight > 0 else d

    # ---- margin space (the local row shard caches its margins, as in the replicated path) ---------------------
    def _gathered_grad(self, f: float, s: float, G: torch.Tensor, w_shard: torch.Tensor, l2_sq: float):
        """(f, gradient slice) from a LOCAL pass result: reduce-scatter G, all-reduce (F, S), then the
        normalization and L2 terms (``l2_sq`` = ||w||^2 of the whole vector)."""
        g_shard = reduce_scatter_full(G.to(torch.float64), self.layout, self.group)
        f, s = _all_reduce_small([f, s], G.device, self.group)
        grad = self._finalize(g_shard, s)
        if self.obj.l2_weight > 0:
            f += 0.5 * self.obj.l2_weight * l2_sq
            grad = grad + self.obj.l2_weight * w_shard
        return f, grad

    def margin_line_search(self, data, x0_shard: torch.Tensor, d_shard: torch.Tensor, t0: float = 1.0,
                           dots=None):
        """:meth:`GLMObjective.margin_line_search` with sharded x0 / d: ONE all-gather of the direction (x0 is
        the accepted point, whose margins the local shard already holds), the direction pass over the local rows,
        then every trial is an elementwise pass + a 2-scalar all-reduce; only the accepted step pays the transpose
        pass and its reduce-scatter. Before this, every trial of the feature-sharded line search was a full
        all-gather + forward + transpose + reduce-scatter."""
        if not hasattr(data, "ls_begin"):
            return None
        norm = self.obj.normalization
        x0 = all_gather_shards(x0_shard, self.layout, self.group)
        d = all_gather_shards(d_shard, self.layout, self.group)
        w0_eff, shift0 = norm.effective(x0)
        d_eff = d * norm.factors.to(d) if norm.factors is not None else d
        d_shift = -float(torch.dot(d_eff, norm.shifts.to(d_eff))) if norm.shifts is not None else 0.0
        if not data.ls_begin(w0_eff, shift0, d_eff, d_shift, t0, self.obj.loss):
            return None
        return ShardedMarginLineSearch(self, data, x0_shard, d_shard, x0, d, dots)

    # TRON trial point from margins (GLMObjective.step_begin / step_add / calculate_step)
    def step_begin(self, data, w_shard: torch.Tensor) -> bool:
        if not hasattr(data, "step_begin"):
            return False
        w_eff, shift = self.obj.normalization.effective(all_gather_shards(w_shard, self.layout, self.group))
        return bool(data.step_begin(w_eff, shift))

    def step_add(self, data, alpha: float):
        data.step_add(alpha)

    def calculate_step(self, data, w_shard: torch.Tensor):
        self.n_value_grad += 1
        norm = self.obj.normalization
        w = all_gather_shards(w_shard, self.layout, self.group)
        w_eff, shift = norm.effective(w)
        f, s, G = data.ls_finish_sums(self.obj.loss, 1.0, w_eff, shift, norm.shifts is not None)
        return self._gathered_grad(f, s, G, w_shard, float(torch.dot(w, w)) if self.obj.l2_weight > 0 else 0.0)


class ShardedMarginLineSearch:
    """phi(t) = F(x0 + t d) with sharded x0 / d (see :class:`photon_ml_amd.function.objective.MarginLineSearch`):
    trials from the local cached margins + one all-reduce of (F, phi') each; ``a, b, c`` = x0.x0, x0.d, d.d of the
    whole vectors (the caller's global dots, or from the gathered vectors: no collective)."""

    def __init__(self, sobj: FeatureShardedObjective, data, x0_shard, d_shard, x0, d, dots=None):
        from ..function.objective import DEFERRED_DOTS
        self.sobj, self.data = sobj, data
        self.x0_shard, self.d_shard = x0_shard, d_shard
        self.l2 = sobj.obj.l2_weight
        if self.l2 > 0 and dots is not DEFERRED_DOTS:
            self.a, self.b, self.c = dots if dots is not None else torch.stack(
                [torch.dot(x0, x0), torch.dot(x0, d), torch.dot(d, d)]).tolist()
        self._x0, self._d = x0, d

    def eval(self, t: float):
        f, dd = self.data.ls_eval(self.sobj.obj.loss, t)
        f, dd = _all_reduce_small([f, dd], self._d.device, self.sobj.group)
        if self.l2 > 0:
            f += 0.5 * self.l2 * (self.a + 2.0 * t * self.b + t * t * self.c)
            dd += self.l2 * (self.b + t * self.c)
        return f, dd

    def finish(self, t: float):
        """(x(t) slice, f(x(t)), gradient slice at x(t)): one transpose pass + its reduce-scatter."""
        so = self.sobj
        so.n_value_grad += 1
        x_shard = self.x0_shard + t * self.d_shard
        x = self._x0 + t * self._d
        norm = so.obj.normalization
        w_eff, shift = norm.effective(x)
        f, s, G = self.data.ls_finish_sums(so.obj.loss, t, w_eff, shift, norm.shifts is not None)
        l2_sq = (self.a + 2.0 * t * self.b + t * t * self.c) if self.l2 > 0 else 0.0
        f, grad = so._gathered_grad(f, s, G, x_shard, l2_sq)
        return x_shard, f, grad


def optimize_feature_sharded(optimizer, objective: GLMObjective, data, initial: Optional[torch.Tensor] = None,
                             normalization: Optional[NormalizationContext] = None, group=None):
    """Run ``optimizer`` (L-BFGS / OWL-QN / TRON, built WITHOUT normalization or box constraints) with the
    optimizer state sharded over features. ``data``: this rank's row shard (all D columns). ``initial``: full
    ORIGINAL-space start (zeros if None). Returns (full ORIGINAL-space coefficients on every rank, final value,
    the sharded objective)."""
    if optimizer.constraints:
        raise ValueError("box constraints are not supported with feature-sharded optimizer state")
    norm = normalization or objective.normalization or no_normalization()
    dim = data.dim
    dev = getattr(data, "device", torch.device("cpu"))
    layout = FeatureShardLayout.current(dim, group)
    w0 = torch.zeros(dim, dtype=torch.float64, device=dev) if initial is None else initial.to(dev, torch.float64)
    w0 = norm.model_to_transformed_space(w0)
    sobj = FeatureShardedObjective(objective, layout, group)
    if hasattr(data, "track_hessian") and getattr(optimizer, "needs_hessian", False):
        data.track_hessian = True
    with active_space(ShardedSpace(group)):
        w_t, f = optimizer.optimize(sobj, data, layout.slice(w0).clone())
        w_full = all_gather_shards(w_t, layout, group)
    return norm.model_to_original_space(w_full), f, sobj

