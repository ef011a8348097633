"""Hyper-parameter search: Sobol random search and Gaussian-process Bayesian search.

Reference: ``photon-lib/.../hyperparameter/`` —
  * ``search/RandomSearch.scala:30-133`` (Sobol candidates scaled into the per-dimension ranges; ``find(n)`` and
    ``find(n, observations)`` with prior observations),
  * ``search/GaussianProcessSearch.scala:55-164`` (after more observations than parameters: fit a GP with a
    Matern 5/2 kernel on the observations, score a pool of 250 Sobol candidates with Expected Improvement and take
    the best; fall back to random search before that),
  * ``estimators/GaussianProcessEstimator.scala:38-148`` (label centring, kernel length scales sampled by slice
    sampling from the GP log-likelihood: burn-in 100, 100 samples; predictions averaged over the sampled kernels),
  * ``estimators/GaussianProcessModel.scala`` (GPML Alg. 2.1), ``estimators/kernels/{RBF,Matern52}.scala``,
  * ``criteria/{ExpectedImprovement,ConfidenceBound}.scala``, ``SliceSampler.scala:53-212``,
    ``Linalg.scala`` (Cholesky solves — host LAPACK via numpy/scipy here: these matrices are tiny).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
from scipy.linalg import cho_factor, cho_solve, cholesky
from scipy.stats import norm, qmc

JITTER = 1e-10


@dataclass(frozen=True)
class DoubleRange:
    start: float
    end: float

    def __post_init__(self):
        if self.start > self.end:
            raise ValueError(f"Invalid range [{self.start}, {self.end}]")

    @staticmethod
    def parse(s: str) -> "DoubleRange":
        """``1e-4-1e4`` style (RANGE_DELIMITER '-' not part of an exponent)."""
        s = s.strip()
        for i in range(1, len(s)):
            if s[i] == "-" and s[i - 1] not in "eE":
                return DoubleRange(float(s[:i]), float(s[i + 1:]))
        raise ValueError(f"cannot parse range {s!r}")


# ---------------------------------------------------------------- kernels
class StationaryKernel:
    def __init__(self, length_scale=(1.0,), bounds=(1e-5, 1e5)):
        self.length_scale = np.atleast_1d(np.asarray(length_scale, dtype=np.float64))
        self.bounds = bounds

    def _ls(self, d):
        return self.length_scale if self.length_scale.size == d else np.full(d, self.length_scale[0])

    def sq_dists(self, a, b=None):
        ls = self._ls(a.shape[1])
        a = a / ls
        b = a if b is None else b / ls
        d = (a * a).sum(1)[:, None] + (b * b).sum(1)[None, :] - 2 * a @ b.T
        return np.maximum(d, 0.0)

    def __call__(self, a, b=None):
        return self.from_sq_dists(self.sq_dists(a, b))

    def params(self):
        return np.log(self.length_scale)

    def param_bounds(self):
        return math.log(self.bounds[0]), math.log(self.bounds[1])

    def expand(self, p, d):
        p = np.atleast_1d(p)
        return p if p.size == d else np.full(d, p[0])

    def with_params(self, theta):
        return type(self)(np.exp(theta), self.bounds)


class RBF(StationaryKernel):
    def from_sq_dists(self, d):
        return np.exp(-0.5 * d)


class Matern52(StationaryKernel):
    def from_sq_dists(self, d):
        f = np.sqrt(5.0 * d)
        return (1.0 + f + 5.0 * d / 3.0) * np.exp(-f)


# ---------------------------------------------------------------- criteria
class ExpectedImprovement:
    def __init__(self, higher_is_better: bool, best: float):
        self.direction = 1.0 if higher_is_better else -1.0
        self.best = best

    def __call__(self, mean, var):
        std = np.sqrt(np.maximum(var, 1e-300))
        gamma = (mean - self.best) / std * self.direction
        return std * (gamma * norm.cdf(gamma) + norm.pdf(gamma))


class ConfidenceBound:
    def __init__(self, higher_is_better: bool, exploration: float = 2.0):
        self.higher = higher_is_better
        self.k = exploration

    def __call__(self, mean, var):
        cb = self.k * np.sqrt(np.maximum(var, 0))
        return mean + cb if self.higher else mean - cb


# ---------------------------------------------------------------- slice sampler
class SliceSampler:
    """Univariate slice sampling along random directions (Neal 2003), stepping out + shrinkage."""

    def __init__(self, logp: Callable, bounds: Tuple[float, float], step: float = 1.0, max_steps: int = 100,
                 seed: int = 0):
        self.logp = logp
        self.lo, self.hi = min(bounds), max(bounds)
        self.step = step
        self.max_steps = max_steps
        self.rng = np.random.default_rng(seed)

    def _inside(self, x):
        return bool(np.all(x >= self.lo) and np.all(x <= self.hi))

    def _lp(self, x):
        return self.logp(x) if self._inside(x) else -np.inf

    def draw(self, x):
        x = np.asarray(x, dtype=np.float64)
        lp0 = self._lp(x)
        if not np.isfinite(lp0):
            return x
        direction = self.rng.normal(size=x.shape)
        direction /= np.linalg.norm(direction)
        y = lp0 + math.log(self.rng.random() + 1e-300)
        u = self.rng.random() * self.step
        lo, hi = -u, self.step - u
        for _ in range(self.max_steps):
            if self._lp(x + lo * direction) <= y:
                break
            lo -= self.step
        for _ in range(self.max_steps):
            if self._lp(x + hi * direction) <= y:
                break
            hi += self.step
        for _ in range(self.max_steps):
            t = lo + self.rng.random() * (hi - lo)
            xn = x + t * direction
            if self._lp(xn) > y:
                return xn
            if t < 0:
                lo = t
            else:
                hi = t
        return x


# ---------------------------------------------------------------- GP
class GaussianProcessModel:
    def __init__(self, x, y, y_mean, kernels, transformation=None):
        self.x, self.y, self.y_mean = x, y, y_mean
        self.kernels = kernels
        self.transformation = transformation
        self.pre = []
        for k in kernels:
            K = k(x) + JITTER * np.eye(len(x))
            L = cholesky(K, lower=True)
            alpha = cho_solve((L, True), y)
            self.pre.append((k, L, alpha))

    def _predict_kernel(self, xs, k, L, alpha):
        kt = k(xs, self.x)
        mean = kt @ alpha + self.y_mean
        v = np.linalg.solve(L, kt.T)
        var = np.diag(k(xs)) - (v * v).sum(0)
        return mean, np.maximum(var, 0.0)

    def predict(self, xs):
        ms, vs = zip(*(self._predict_kernel(xs, *p) for p in self.pre))
        return np.mean(ms, 0), np.mean(vs, 0)

    def predict_transformed(self, xs):
        outs = []
        for p in self.pre:
            m, v = self._predict_kernel(xs, *p)
            outs.append(self.transformation(m, v) if self.transformation else m)
        return np.mean(outs, 0)


class GaussianProcessEstimator:
    def __init__(self, kernel=None, normalize_labels=False, transformation=None, burn_in: int = 100,
                 n_samples: int = 100, seed: int = 0):
        self.kernel = kernel or RBF()
        self.normalize_labels = normalize_labels
        self.transformation = transformation
        self.burn_in, self.n_samples = burn_in, n_samples
        self.seed = seed

    def log_likelihood(self, x, y, theta):
        K = self.kernel.with_params(theta)(x) + JITTER * np.eye(len(x))
        try:
            L = cholesky(K, lower=True)
        except np.linalg.LinAlgError:
            return -np.inf
        alpha = cho_solve((L, True), y)
        return float(-0.5 * y @ alpha - np.log(np.diag(L)).sum() - len(x) / 2.0 * math.log(2 * math.pi))

    def fit(self, x, y) -> GaussianProcessModel:
        x = np.asarray(x, dtype=np.float64)
        y = np.asarray(y, dtype=np.float64)
        m = float(y.mean()) if self.normalize_labels else 0.0
        yt = y - m
        sampler = SliceSampler(lambda th: self.log_likelihood(x, yt, th), self.kernel.param_bounds(), seed=self.seed)
        th = self.kernel.expand(self.kernel.params(), x.shape[1])
        for _ in range(self.burn_in):
            th = sampler.draw(th)
        samples = []
        for _ in range(self.n_samples):
            th = sampler.draw(th)
            samples.append(self.kernel.with_params(th))
        return GaussianProcessModel(x, yt, m, samples, self.transformation)


# ---------------------------------------------------------------- searches
class EvaluationFunction:
    """Maps a candidate vector to (evaluation value, observation) — see EvaluationFunction.scala."""

    higher_is_better = True

    def __call__(self, candidate: np.ndarray):
        raise NotImplementedError

    def vectorize_params(self, observation) -> np.ndarray:
        raise NotImplementedError

    def get_evaluation_value(self, observation) -> float:
        raise NotImplementedError


class RandomSearch:
    def __init__(self, ranges: Sequence[DoubleRange], evaluation_function: EvaluationFunction, seed: int = 0):
        self.ranges = list(ranges)
        self.fn = evaluation_function
        self.n_params = len(self.ranges)
        self.sobol = qmc.Sobol(d=self.n_params, scramble=False)
        if seed:
            self.sobol.fast_forward(int(seed) % (2 ** 20))
        self.seed = seed

    def draw_candidates(self, n: int) -> np.ndarray:
        c = self.sobol.random(n)
        for j, r in enumerate(self.ranges):
            c[:, j] = c[:, j] * (r.end - r.start) + r.start
        return c

    def next(self, last_candidate, last_value) -> np.ndarray:
        return self.draw_candidates(1)[0]

    def on_observation(self, point, value):
        pass

    def find(self, n: int, observations: Sequence = ()) -> List:
        if n <= 0:
            raise ValueError("The number of results must be greater than zero.")
        results = []
        if observations:
            conv = [(self.fn.vectorize_params(o), self.fn.get_evaluation_value(o)) for o in observations]
            for c, v in conv[:-1]:
                self.on_observation(c, v)
            last = conv[-1]
        else:
            cand = self.draw_candidates(1)[0]
            value, obs = self.fn(cand)
            results.append(obs)
            last = (cand, value)
            n -= 1
        for _ in range(n):
            cand = self.next(*last)
            value, obs = self.fn(cand)
            results.append(obs)
            last = (cand, value)
        return results


class GaussianProcessSearch(RandomSearch):
    def __init__(self, ranges, evaluation_function, higher_is_better: Optional[bool] = None,
                 candidate_pool_size: int = 250, seed: int = 0, burn_in: int = 100, n_samples: int = 100):
        super().__init__(ranges, evaluation_function, seed)
        self.higher = evaluation_function.higher_is_better if higher_is_better is None else higher_is_better
        self.pool = candidate_pool_size
        self.points: List[np.ndarray] = []
        self.evals: List[float] = []
        self.best = -np.inf if self.higher else np.inf
        self.burn_in, self.n_samples = burn_in, n_samples
        self.last_model = None

    def on_observation(self, point, value):
        self.points.append(np.asarray(point, dtype=np.float64))
        self.evals.append(float(value))
        if (value > self.best) if self.higher else (value < self.best):
            self.best = float(value)

    def next(self, last_candidate, last_value):
        self.on_observation(last_candidate, last_value)
        if len(self.points) > self.n_params:
            cands = self.draw_candidates(self.pool)
            est = GaussianProcessEstimator(Matern52(), True, ExpectedImprovement(self.higher, self.best),
                                           self.burn_in, self.n_samples, seed=self.seed)
            model = est.fit(np.stack(self.points), np.array(self.evals))
            self.last_model = model
            pred = model.predict_transformed(cands)
            return cands[int(np.argmax(pred))]  # EI is maximised in both directions
        return super().next(last_candidate, last_value)
