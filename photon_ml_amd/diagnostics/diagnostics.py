"""Model and training diagnostics for the legacy GLM driver.

Reference (``photon-diagnostics/src/main/scala/com/linkedin/photon/ml/``):

* ``diagnostics/hl/*`` — Hosmer–Lemeshow goodness of fit for logistic models: equal-width probability bins
  (count = min(dim + 2, 0.9·sqrt(n) + 0.9·log1p(n)) — the reference multiplies BOTH terms by factor A, kept),
  χ² = Σ (obs−exp)²/exp over positive and negative counts, dof = bins − 2, cut-offs at standard confidence
  levels, warnings when an expected count is below 5.
* ``diagnostics/independence/*`` — Kendall τ between prediction and error on a ≤ 5000-sample subset:
  concordant / discordant / tie counts, τ-a, τ-b, z-score, two-sided p-value (``KendallTauAnalysis.scala``).
* ``diagnostics/featureimportance/*`` — |w_j|·E|x_j| (expected magnitude) and |w_j|·Var(x_j) (variance)
  importances; top-50 ranked features and the importance at 100 fractiles.
* ``diagnostics/fitting/FittingDiagnostic.scala`` — learning curves: hold out 1/10 of the samples, train on
  growing 1/10 portions (warm-started), evaluate train + hold-out metrics (skipped with < 10·dim samples).
* ``BootstrapTraining.scala`` + ``diagnostics/bootstrap/BootstrapTrainingDiagnostic.scala`` — 15 bootstrap
  fits on 70 % (≤ 90 %) tag splits, per-coefficient and per-metric min/Q1/median/Q3/max, important features and
  coefficients whose inter-quartile range straddles 0.

Sampling uses numpy's PCG64 (the reference uses MersenneTwister), so individual splits differ; the statistics
themselves follow the reference formulas.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
from scipy.stats import chi2, norm

from ..constants import split_feature_key
from ..data.matrix import LabeledData
from ..models.glm import GeneralizedLinearModel, LogisticRegressionModel
from .evaluation import MetricsMap, evaluate


def _scores(model: GeneralizedLinearModel, data: LabeledData, with_offset: bool = True) -> np.ndarray:
    w = model.coefficients.means.detach().cpu().numpy()
    z = np.asarray(data.x @ w).ravel()
    if with_offset:
        z = z + data.offsets
    import torch
    return model.mean_from_score(torch.from_numpy(z)).numpy()


# ------------------------------------------------------------------------------------------------ Hosmer-Lemeshow
STANDARD_CONFIDENCE_LEVELS = [0.000001, 0.01, 0.05, 0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 0.9, 0.95, 0.99, 0.999999]
MINIMUM_EXPECTED_IN_BUCKET = 5
DATA_HEURISTIC_FACTOR_A = 0.9


@dataclass
class HistogramBin:
    lower: float
    upper: float
    observed_pos: int = 0
    observed_neg: int = 0

    @property
    def expected_pos(self) -> int:
        """ceil(count * bin-centre probability), as PredictedProbabilityVersusObservedFrequencyHistogramBin."""
        return int(math.ceil((self.observed_pos + self.observed_neg) * 0.5 * (self.lower + self.upper)))

    @property
    def expected_neg(self) -> int:
        return (self.observed_pos + self.observed_neg) - self.expected_pos

    def __str__(self):
        return (f"[{self.lower:.3f}, {self.upper:.3f}): observed pos={self.observed_pos} neg={self.observed_neg}, "
                f"expected pos={self.expected_pos} neg={self.expected_neg}")


@dataclass
class HosmerLemeshowReport:
    binning_msg: str
    chi_square_msg: str
    chi_squared_score: float
    degrees_of_freedom: int
    chi_squared_prob: float
    cutoffs: List[Tuple[float, float]]
    histogram: List[HistogramBin]

    def test_description(self) -> str:
        return f"Chi^2 = [{self.chi_squared_score:.6f}] on [{self.degrees_of_freedom}] degrees of freedom"

    def point_probability(self) -> str:
        return f"Pr[Chi^2 < {self.chi_squared_score}] = [{100.0 * self.chi_squared_prob:.9g}%]"

    def __str__(self):
        cut = "\n".join(f"  Pr[X <= {c:12.9f}] at confidence {100 * (1 - p):.6f}%: "
                        f"{'reject' if self.chi_squared_score > c else 'accept'} fit" for p, c in self.cutoffs)
        hist = "\n    ".join(str(b) for b in self.histogram)
        return f"{self.test_description()}\n{self.point_probability()}\nCutoffs:\n{cut}\nHistogram:\n    {hist}"


def hl_bin_count(n: int, dim: int) -> Tuple[str, int]:
    by_dim = dim + 2
    by_data = int(DATA_HEURISTIC_FACTOR_A * math.sqrt(n) + DATA_HEURISTIC_FACTOR_A * math.log1p(n))
    bins = max(1, min(by_dim, by_data))
    ok = "Sufficient bins for a discriminative test" if bins >= by_dim else (
        "Not enough bins for a discriminative test; please be careful when interpreting these results or rerun "
        "with more data")
    msg = (f"Number of test set samples: {n}\nSample dimensionality: {dim}\n"
           f"Target number of bins based on dimensionality alone: {by_dim}\n"
           f"Target number of bins based on data alone: {by_data}\n{ok}")
    return msg, bins


def hosmer_lemeshow(labels: np.ndarray, probs: np.ndarray, dim: int) -> HosmerLemeshowReport:
    probs = np.asarray(probs, dtype=np.float64)
    if ((probs < 0) | (probs > 1)).any():
        raise ValueError("predicted probabilities must lie in [0, 1]")
    msg, nb = hl_bin_count(len(probs), dim)
    edges = np.arange(nb + 1) / nb
    idx = np.minimum((probs * nb).astype(np.int64), nb - 1)
    pos = np.abs(np.asarray(labels) - 1.0) < 1e-12
    n_pos = np.bincount(idx[pos], minlength=nb)
    n_neg = np.bincount(idx[~pos], minlength=nb)
    bins = [HistogramBin(edges[i], edges[i + 1], int(n_pos[i]), int(n_neg[i])) for i in range(nb)]
    chi, notes = 0.0, []
    for b in bins:
        if b.expected_pos > 0:
            chi += (b.observed_pos - b.expected_pos) ** 2 / b.expected_pos
        if b.expected_pos < MINIMUM_EXPECTED_IN_BUCKET:
            notes.append(f"For bin [{b}], expected positive count is too small to soundly use in a Chi^2 estimate")
        if b.expected_neg > 0:
            chi += (b.observed_neg - b.expected_neg) ** 2 / b.expected_neg
        if b.expected_neg < MINIMUM_EXPECTED_IN_BUCKET:
            notes.append(f"For bin [{b}], expected negative count is too small to soundly use in a Chi^2 estimate")
    dof = nb - 2
    if dof > 0:
        cutoffs = [(p, float(chi2.ppf(p, dof))) for p in STANDARD_CONFIDENCE_LEVELS]
        prob = float(chi2.cdf(chi, dof))
    else:
        cutoffs, prob = [], float("nan")
    return HosmerLemeshowReport(msg, "\n".join(notes), chi, dof, prob, cutoffs, bins)


# ------------------------------------------------------------------------------------------------ Kendall tau
@dataclass
class KendallTauReport:
    concordant: int
    discordant: int
    n_items: int
    n_pairs: int
    effective_pairs: int
    tau_alpha: float
    tau_beta: float
    z_alpha: float
    p_value: float
    message: str = ""


def kendall_tau(a: np.ndarray, b: np.ndarray) -> KendallTauReport:
    """O(n^2) pair classification on the (already sub-sampled) arrays, vectorised in row blocks."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    n = len(a)
    conc = disc = ties_a = ties_b = 0
    for i0 in range(0, n, 1024):
        ai, bi = a[i0:i0 + 1024, None], b[i0:i0 + 1024, None]
        j = np.arange(n)[None, :]
        upper = j > np.arange(i0, min(n, i0 + 1024))[:, None]
        da, db = np.sign(ai - a[None, :]), np.sign(bi - b[None, :])
        conc += int(((da * db > 0) & upper).sum())
        disc += int(((da * db < 0) & upper).sum())
        ties_a += int(((da == 0) & upper).sum())
        ties_b += int(((da != 0) & (db == 0) & upper).sum())
    pairs = n * (n - 1) // 2
    eff = conc + disc
    tau_a = (conc - disc) / eff if eff else float("nan")
    tau_b = (conc - disc) / math.sqrt(max(1, (pairs - ties_a)) * max(1, (pairs - ties_b)))
    aa = 2.0 * (2.0 * n + 5.0)
    bb = 9.0 * n * (n - 1)
    d = math.sqrt(aa / bb) if bb > 0 else 1.0
    z = tau_a / d if eff else float("nan")
    p = float(norm.cdf(abs(z)) - norm.cdf(-abs(z))) if eff else float("nan")
    msg = ""
    if ties_a + ties_b > 0:
        msg = (f"Note: detected ties (ties in first variable: {ties_a}, ties in second variable: {ties_b}). The z "
               "score / p value for tau-alpha over-estimate the degree of independence.")
    return KendallTauReport(conc, disc, n, pairs, eff, tau_a, tau_b, z, p, msg)


@dataclass
class PredictionErrorIndependenceReport:
    errors: np.ndarray
    predictions: np.ndarray
    kendall_tau: KendallTauReport


MAXIMUM_SAMPLE_SIZE = 5000


def prediction_error_independence(model, data: LabeledData, seed: int = 0) -> PredictionErrorIndependenceReport:
    pred = _scores(model, data)
    err = data.y - pred
    rng = np.random.default_rng(seed)
    idx = rng.choice(len(pred), size=min(MAXIMUM_SAMPLE_SIZE, len(pred)), replace=False)
    return PredictionErrorIndependenceReport(err[idx], pred[idx], kendall_tau(pred[idx], err[idx]))


# ------------------------------------------------------------------------------------------------ importance
MAX_RANKED_FEATURES = 50
NUM_IMPORTANCE_FRACTILES = 100


@dataclass
class FeatureImportanceReport:
    importance_type: str
    importance_description: str
    feature_importance: Dict[Tuple[str, str], Tuple[int, float, str]]
    rank_to_importance: Dict[float, float]


def feature_importance(model, index_map, summary=None, kind: str = "magnitude") -> FeatureImportanceReport:
    w = model.coefficients.means.detach().cpu().numpy()
    d = len(w)
    if kind == "magnitude":
        scale = summary.mean_abs.numpy() if summary is not None else np.ones(d)
        typ = "Inner product expectation"
        desc = "Expected magnitude of inner product contribution" if summary is not None else \
            "Magnitude of feature coefficient"
    else:
        scale = summary.variance.numpy() if summary is not None else np.ones(d)
        typ = "Inner product variance"
        desc = "Expected inner product variance contribution" if summary is not None else \
            "Magnitude of feature coefficient"
    imp = np.abs(w * scale)
    order = np.argsort(-imp, kind="stable")
    ranked = [(j, float(imp[j])) for j in order]
    fractiles = {}
    if ranked:
        for q in range(NUM_IMPORTANCE_FRACTILES + 1):
            k = min(len(ranked) - 1, q * len(ranked) // MAX_RANKED_FEATURES)
            fractiles[100.0 * q / NUM_IMPORTANCE_FRACTILES] = ranked[k][1]
    feats = {}
    for j, v in ranked[:MAX_RANKED_FEATURES]:
        key = index_map.get_feature_name(int(j)) if index_map is not None else None
        nt = split_feature_key(key) if key else (str(j), "")
        text = f"Feature (name=[{nt[0]}], term=[{nt[1]}]) importance = [{v:.3f}], coefficient = [{w[j]:.6g}]"
        if summary is not None:
            text += (f" min=[{float(summary.min[j])}], mean=[{float(summary.mean[j])}], "
                     f"max=[{float(summary.max[j])}], variance=[{float(summary.variance[j])}]")
        feats[nt] = (int(j), v, text)
    return FeatureImportanceReport(typ, desc, feats, fractiles)


# ------------------------------------------------------------------------------------------------ learning curves
NUM_TRAINING_PARTITIONS = 10
MIN_SAMPLES_PER_PARTITION_PER_DIMENSION = 10


@dataclass
class FittingReport:
    metrics: Dict[str, Tuple[np.ndarray, np.ndarray, np.ndarray]]  # metric -> (portions %, train, test)
    message: str = ""


TrainFunc = Callable[[LabeledData, Dict[float, GeneralizedLinearModel]], List[Tuple[float, GeneralizedLinearModel]]]


def fitting_diagnostic(train_func: TrainFunc, warm_start: Dict[float, GeneralizedLinearModel], data: LabeledData,
                       seed: int = 0) -> Dict[float, FittingReport]:
    n, dim = data.n_rows, data.n_features
    if n <= dim * MIN_SAMPLES_PER_PARTITION_PER_DIMENSION:
        return {}
    tags = np.random.default_rng(seed).integers(0, NUM_TRAINING_PARTITIONS, size=n)
    hold = data.subset(np.nonzero(tags == NUM_TRAINING_PARTITIONS - 1)[0])
    curves: Dict[float, Dict[str, list]] = {}
    prev = dict(warm_start)
    for max_tag in range(NUM_TRAINING_PARTITIONS - 1):
        part = data.subset(np.nonzero(tags <= max_tag)[0])
        portion = 100.0 * part.n_rows / n
        models = dict(train_func(part, prev))
        prev = models
        for lam, m in models.items():
            test, train = evaluate(m, hold), evaluate(m, part)
            c = curves.setdefault(lam, {})
            for k, v in test.items():
                c.setdefault(k, []).append((portion, train[k], v))
    out = {}
    for lam, c in curves.items():
        out[lam] = FittingReport({k: tuple(np.array(col) for col in zip(*sorted(v))) for k, v in c.items()})
    return out


# ------------------------------------------------------------------------------------------------ bootstrap
@dataclass
class CoefficientSummary:
    values: List[float] = field(default_factory=list)

    def accumulate(self, x: float):
        self.values.append(float(x))

    def _sorted(self):
        return sorted(self.values)

    @property
    def count(self):
        return len(self.values)

    @property
    def mean(self):
        return float(np.mean(self.values))

    @property
    def std(self):
        return float(np.std(self.values, ddof=1)) if len(self.values) > 1 else 0.0

    @property
    def min(self):
        return min(self.values)

    @property
    def max(self):
        return max(self.values)

    def first_quartile(self):
        s = self._sorted()
        return s[len(s) // 4]

    def median(self):
        s = self._sorted()
        return s[2 * len(s) // 4]

    def third_quartile(self):
        s = self._sorted()
        return s[3 * len(s) // 4]

    def __str__(self):
        return (f"Range: [Min: {self.min:.3f}, Q1: {self.first_quartile():.3f}, Med: {self.median():.3f}, "
                f"Q3: {self.third_quartile():.3f}, Max: {self.max:.3f}) Mean: [{self.mean:.3f}], "
                f"Std. Dev.[{self.std:.3f}], # samples = [{self.count}]")


@dataclass
class BootstrapReport:
    metric_distributions: Dict[str, Tuple[float, float, float, float, float]]
    important_features: Dict[Tuple[str, str], CoefficientSummary]
    zero_crossing_features: Dict[Tuple[str, str], Tuple[int, float, CoefficientSummary]]


NUM_IMPORTANT_FEATURES = 15
DEFAULT_BOOTSTRAP_SAMPLES = 15
DEFAULT_BOOTSTRAP_PORTION = 0.7


def bootstrap_training(train_func: TrainFunc, warm_start, data: LabeledData, n_samples: int = DEFAULT_BOOTSTRAP_SAMPLES,
                       portion: float = DEFAULT_BOOTSTRAP_PORTION, seed: int = 0):
    """BootstrapTraining.bootstrap: returns lambda -> list of (model, hold-out metrics)."""
    if n_samples <= 1:
        raise ValueError(f"Number of bootstrap samples must be at least 2, got [{n_samples}]")
    if not 0 < portion <= 1:
        raise ValueError(f"Portion of training samples must be in (0, 1], got [{portion}]")
    n_splits = 1000
    target = min(900, int(portion * n_splits))
    rng = np.random.default_rng(seed)
    tags = rng.integers(0, n_splits, size=data.n_rows)
    out: Dict[float, list] = {}
    for _ in range(n_samples):
        shuffled = rng.permutation(n_splits)
        train_tags = np.zeros(n_splits, dtype=bool)
        train_tags[shuffled[:target]] = True
        tr = data.subset(np.nonzero(train_tags[tags])[0])
        ho = data.subset(np.nonzero(~train_tags[tags])[0])
        for lam, m in train_func(tr, warm_start):
            out.setdefault(lam, []).append((m, evaluate(m, ho)))
    return out


def bootstrap_diagnostic(train_func: TrainFunc, models: Dict[float, GeneralizedLinearModel], data: LabeledData,
                         index_map, summary=None, n_samples: int = DEFAULT_BOOTSTRAP_SAMPLES,
                         portion: float = DEFAULT_BOOTSTRAP_PORTION, seed: int = 0) -> Dict[float, BootstrapReport]:
    runs = bootstrap_training(train_func, models, data, n_samples, portion, seed)
    reports = {}
    for lam, mm in runs.items():
        d = mm[0][0].coefficients.dim
        coeffs = [CoefficientSummary() for _ in range(d)]
        for m, _ in mm:
            for j, v in enumerate(m.coefficients.means.detach().cpu().numpy()):
                coeffs[j].accumulate(v)
        metrics: Dict[str, CoefficientSummary] = {}
        for _, met in mm:
            for k, v in met.items():
                metrics.setdefault(k, CoefficientSummary()).accumulate(v)
        scale = summary.mean_abs.numpy() if summary is not None else np.ones(d)
        w = models[lam].coefficients.means.detach().cpu().numpy() if lam in models else np.ones(d)
        imp = scale * np.abs(w)

        def name(j):
            key = index_map.get_feature_name(j) if index_map is not None else None
            return split_feature_key(key) if key else (str(j), "")
        order = np.argsort(imp, kind="stable")
        important = {name(int(j)): coeffs[int(j)] for j in order[-NUM_IMPORTANT_FEATURES:]}
        straddle = {name(j): (j, float(imp[j]), coeffs[j]) for j in range(d)
                    if coeffs[j].first_quartile() < 0 < coeffs[j].third_quartile()}
        metric_dist = {k: (s.min, s.first_quartile(), s.median(), s.third_quartile(), s.max) for k, s in metrics.items()}
        reports[lam] = BootstrapReport(metric_dist, important, straddle)
    return reports


# ------------------------------------------------------------------------------------------------ model report
@dataclass
class ModelDiagnosticReport:
    model: GeneralizedLinearModel
    lam: float
    description: str
    metrics: MetricsMap
    summary: object = None
    prediction_error_independence: Optional[PredictionErrorIndependenceReport] = None
    hosmer_lemeshow: Optional[HosmerLemeshowReport] = None
    mean_impact_importance: Optional[FeatureImportanceReport] = None
    variance_impact_importance: Optional[FeatureImportanceReport] = None
    fit_report: Optional[FittingReport] = None
    bootstrap_report: Optional[BootstrapReport] = None


def validation_diagnostics(model, lam, data: LabeledData, index_map, summary=None, metrics=None,
                           seed: int = 0) -> ModelDiagnosticReport:
    hl = None
    if isinstance(model, LogisticRegressionModel):
        hl = hosmer_lemeshow(data.y, _scores(model, data, with_offset=False), data.n_features)
    return ModelDiagnosticReport(
        model, lam, f"{type(model).__name__} @ lambda = {lam}", metrics or evaluate(model, data), summary,
        prediction_error_independence(model, data, seed), hl,
        feature_importance(model, index_map, summary, "magnitude"),
        feature_importance(model, index_map, summary, "variance"))
