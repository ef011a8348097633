"""photon_ml_amd — an MI355X-native GLM + GAME (GLMix) training engine with Photon ML's capabilities.

Layout (see SURVEY.md §1 for the reference layer map):
  ops/            HIP/CDNA4 kernels (C ABI runtime in ops/csrc) + fp64 torch reference backend
  function/       pointwise losses and GLM objectives (normalisation folding, L2)
  optimization/   L-BFGS, OWL-QN, TRON, Photon convergence logic, configs, optimisation problems
  normalization/  NormalizationContext
  stat/           feature statistics
  data/           labeled data, GAME datasets (fixed/random effect), synthetic generators, readers
  models/         GLM model classes, coefficients, fixed/random-effect models, GameModel
  algorithm/      GAME coordinates and coordinate descent
  estimators/     GameEstimator / GameTransformer / GLM lambda-path training
  evaluation/     evaluators (AUC, RMSE, losses, per-group AUC / precision@k)
  sampling/       down-samplers
  projector/      random-effect projectors (index map, random Gaussian, identity)
  parallel/       torch.distributed (RCCL over xGMI) process groups, sharding, all-to-all routing
  io/             Avro OCF codec (native), model/score/feature-stat IO, index maps, LibSVM
  cli/            Driver / GameTrainingDriver / GameScoringDriver / FeatureIndexingDriver / feature bags
  hyperparameter/ Sobol random search, Gaussian-process Bayesian search
  diagnostics/    metrics, bootstrap, fitting curves, Hosmer-Lemeshow, Kendall tau, feature importance, reports
  utils/          logging, timing, events, checkpointing
"""
__version__ = "0.1.0"
