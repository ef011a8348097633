"""Worker bodies for the multi-process (gloo, CPU) tests in test_distributed.py — the analogue of the
reference's Spark local[*] "fake cluster" tests (SURVEY §4 tier 4)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _init(rank, world, port):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank), "PML_BACKEND": "torch"})
    from photon_ml_amd.parallel.dist import init_distributed
    init_distributed("gloo")


def glm_worker(rank, world, port, out):
    _init(rank, world, port)
    from photon_ml_amd.data.synthetic import generate_glm_data
    from photon_ml_amd.estimators.game_estimator import train_generalized_linear_model
    from photon_ml_amd.optimization.config import RegularizationContext
    data, _ = generate_glm_data("LOGISTIC_REGRESSION", 3000, 40, density=0.2, seed=7)
    local = data.subset(np.arange(rank, data.n_rows, world))
    for opt, reg in (("LBFGS", "L2"), ("TRON", "L2"), ("LBFGS", "L1")):
        res = train_generalized_linear_model(local, "LOGISTIC_REGRESSION", opt, RegularizationContext(reg), [1.0],
                                             max_iterations=200, tolerance=1e-10, device="cpu")
        np.save(f"{out}/glm_{opt}_{reg}_r{rank}.npy", res[0][1].coefficients.means.numpy())
    import torch.distributed as dist
    dist.destroy_process_group()


def game_worker(rank, world, port, out):
    _init(rank, world, port)
    from photon_ml_amd.data.game_data import generate_game_data
    from photon_ml_amd.data.random_effect import FixedEffectDataConfiguration, RandomEffectDataConfiguration
    from photon_ml_amd.estimators.game_estimator import GameEstimator
    from photon_ml_amd.io.index_map import DefaultIndexMap
    from photon_ml_amd.io.model_io import save_game_model
    from photon_ml_amd.optimization.config import (GLMOptimizationConfiguration, OptimizerConfig,
                                                   RegularizationContext)
    data, _ = generate_game_data(n_rows=3000, n_users=40, n_items=25, seed=31, task="LOGISTIC_REGRESSION")
    tr, va = data.subset(np.arange(2400)), data.subset(np.arange(2400, 3000))
    tr_l = tr.subset(np.arange(rank, tr.n_rows, world))
    va_l = va.subset(np.arange(rank, va.n_rows, world))
    cfg = GLMOptimizationConfiguration(OptimizerConfig("TRON", 50, 1e-10), RegularizationContext("L2"), 1.0)
    est = (GameEstimator(device="cpu").set_training_task("LOGISTIC_REGRESSION")
           .set_coordinate_data_configurations({"global": FixedEffectDataConfiguration("global"),
                                                "per-user": RandomEffectDataConfiguration("userId", "user"),
                                                "per-item": RandomEffectDataConfiguration("itemId", "item")})
           .set_coordinate_update_sequence(["global", "per-user", "per-item"])
           .set_coordinate_descent_iterations(2)
           .set_validation_evaluators(["AUC", "LOGISTIC_LOSS", "AUC:userId"]))
    res = est.fit(tr_l, va_l, [{"global": cfg, "per-user": cfg, "per-item": cfg}])[0]
    np.save(f"{out}/game_fe_r{rank}.npy", res.model.get("global").glm.coefficients.means.numpy())
    np.save(f"{out}/game_eval_r{rank}.npy", np.array([v for _, v in res.evaluations]))
    maps = {s: DefaultIndexMap.from_keys([f"f{j}\u0001t" for j in range(data.shards[s].shape[1])])
            for s in data.shards}
    save_game_model(res.model, f"{out}/model", maps, opt_configs=res.config)
    import torch.distributed as dist
    if dist.is_initialized():      # (not for a plain WORLD_SIZE=1 run)
        dist.barrier()
        dist.destroy_process_group()


def placed_worker(rank, world, port, out):
    """Entity-aligned placement (parallel/placement.py) vs per-update routing: (a) the primary random-effect
    coordinate alone on the same partial scores — bitwise-equal models and scores, zero routed bytes; (b) a whole
    GAME fit with and without placement."""
    _init(rank, world, port)
    import torch
    from photon_ml_amd.algorithm.coordinates import ShardedRandomEffectCoordinate
    from photon_ml_amd.data.game_data import generate_game_data
    from photon_ml_amd.data.random_effect import FixedEffectDataConfiguration, RandomEffectDataConfiguration
    from photon_ml_amd.estimators.game_estimator import GameEstimator
    from photon_ml_amd.optimization.config import (GLMOptimizationConfiguration, OptimizerConfig,
                                                   RegularizationContext)
    from photon_ml_amd.parallel.placement import place_rows_by_entity
    data, _ = generate_game_data(n_rows=3000, n_users=40, n_items=25, seed=31, task="LOGISTIC_REGRESSION")
    tr = data.subset(np.arange(2400))
    tr_l = tr.subset(np.arange(rank, tr.n_rows, world))
    cfg = GLMOptimizationConfiguration(OptimizerConfig("TRON", 50, 1e-10), RegularizationContext("L2"), 1.0)
    dc = RandomEffectDataConfiguration("userId", "user")
    placed = place_rows_by_entity(tr_l, "userId", "cpu")
    assert placed.placement.re_type == "userId"
    # partial scores per ORIGINAL row (deterministic function of the uid), carried to the placed rows by uid
    ps_of = lambda d: torch.from_numpy(np.sin(d.uids.astype(np.float64)) * 0.3)
    res = {}
    for name, d in (("routed", tr_l), ("placed", placed)):
        c = ShardedRandomEffectCoordinate("per-user", d, dc, cfg, "LOGISTIC_REGRESSION", device="cpu")
        assert c.placed == (name == "placed")
        m = c.update_model(c.initialize_model(), ps_of(d))
        s = c.score(m)
        rb = c.routed_bytes
        m2 = c.update_model(m, ps_of(d) * 0.5)
        res[name] = (m2, s, d.uids, rb)
    (ma, sa, ua, rba), (mb, sb, ub, rbb) = res["routed"], res["placed"]
    assert rbb == 0 and (world == 1 or rba > 0), (rba, rbb)
    assert sorted(ma.entity_ids) == sorted(mb.entity_ids)
    for e in ma.entity_ids:
        assert np.array_equal(ma.coefficients_of(e).means.numpy(), mb.coefficients_of(e).means.numpy()), e
    # scores: per uid, bitwise
    sa_by, sb_by = dict(zip(ua.tolist(), sa.numpy().tolist())), dict(zip(ub.tolist(), sb.numpy().tolist()))
    np.save(f"{out}/placed_scores_r{rank}.npy", np.array([[u, sb_by[u]] for u in sorted(sb_by)]))
    np.save(f"{out}/routed_scores_r{rank}.npy", np.array([[u, sa_by[u]] for u in sorted(sa_by)]))
    # (b) whole fits
    for mode in ("auto", None):
        est = (GameEstimator(device="cpu").set_training_task("LOGISTIC_REGRESSION")
               .set_coordinate_data_configurations({"global": FixedEffectDataConfiguration("global"),
                                                    "per-user": dc,
                                                    "per-item": RandomEffectDataConfiguration("itemId", "item")})
               .set_coordinate_update_sequence(["global", "per-user", "per-item"])
               .set_coordinate_descent_iterations(2).set_entity_placement(mode))
        r = est.fit(tr_l, None, [{"global": cfg, "per-user": cfg, "per-item": cfg}])[0]
        tag = "auto" if mode else "none"
        assert est.coordinates["per-user"].placed == (mode == "auto")
        assert not est.coordinates["per-item"].placed
        np.save(f"{out}/fit_{tag}_fe_r{rank}.npy", r.model.get("global").glm.coefficients.means.numpy())
        np.save(f"{out}/fit_{tag}_bytes_r{rank}.npy", np.array([est.coordinates["per-user"].routed_bytes,
                                                               est.coordinates["per-item"].routed_bytes]))
    import torch.distributed as dist
    dist.barrier()
    dist.destroy_process_group()


def sharding_worker(rank, world, port, out):
    _init(rank, world, port)
    import scipy.sparse as sp
    from photon_ml_amd.parallel.sharding import EntityPartitioner, RowRouter, stable_hash64
    rng = np.random.default_rng(rank)
    ids = np.array([f"u{i}" for i in rng.integers(0, 30, 80)], dtype=object)
    keys = stable_hash64(ids)
    part = EntityPartitioner.build(keys, top_k=5)
    router = RowRouter(part.owner(keys))
    v = torch.arange(80, dtype=torch.float64) + 1000 * rank
    assert torch.equal(router.backward(router.forward(v)), v)
    x = sp.random(80, 9, density=0.3, format="csr", random_state=rank)
    assert np.allclose(router.forward_csr(x).toarray(), router.forward(torch.from_numpy(x.toarray())).numpy())
    # every received row belongs to an entity this rank owns
    recv_keys = router.forward(torch.from_numpy(keys)).numpy()
    assert np.all(part.owner(recv_keys) == rank)
    np.save(f"{out}/shard_r{rank}.npy", np.array([router.n_recv]))
    # device data built from DIFFERENT row shards shares one feature order (all-reduced counts), so the bucketed,
    # overlapped gradient all-reduce is enabled for real (CLI / GAME) data, not only for the synthetic bench
    from photon_ml_amd.data.synthetic import generate_glm_data
    from photon_ml_amd.ops.device import DeviceGLMData
    from photon_ml_amd.parallel.dist import DistributedGLMData
    data, _ = generate_glm_data("LOGISTIC_REGRESSION", 2000, 300, density=0.05, seed=3)
    local = data.subset(np.arange(rank, data.n_rows, world))         # different row shards, uneven for world 3, 8
    dev = DeviceGLMData.from_labeled(local, "cpu", "f64", chunk_rows=512, layout="tiled")
    assert DistributedGLMData(dev).overlap
    np.save(f"{out}/perm_r{rank}.npy", dev.old_of_new.numpy())
    import torch.distributed as dist
    dist.destroy_process_group()


def fsdp_worker(rank, world, port, out):
    """Feature-sharded optimizer state (each rank: half the rows, a 1/world slice of w, g and the history)."""
    _init(rank, world, port)
    from photon_ml_amd.data.synthetic import generate_glm_data
    from photon_ml_amd.function.losses import loss_for_task
    from photon_ml_amd.function.objective import GLMObjective
    from photon_ml_amd.normalization.context import NormalizationContext
    from photon_ml_amd.ops.backend import make_glm_data
    from photon_ml_amd.optimization.config import OptimizerConfig, RegularizationContext, build_optimizer
    from photon_ml_amd.parallel.feature_sharding import optimize_feature_sharded
    from photon_ml_amd.stat.summary import BasicStatisticalSummary
    data, _ = generate_glm_data("LOGISTIC_REGRESSION", 3000, 41, density=0.2, seed=7)
    local = data.subset(np.arange(rank, data.n_rows, world))
    gd = make_glm_data(local, "cpu", "f64")
    for opt, reg, norm in (("LBFGS", "L2", None), ("TRON", "L2", None), ("LBFGS", "L1", None),
                           ("LBFGS", "L2", "STANDARDIZATION")):
        rc = RegularizationContext(reg)
        nc = None
        if norm:
            nc = NormalizationContext.build(norm, BasicStatisticalSummary.compute(data.x), data.n_features - 1)
        obj = GLMObjective(loss_for_task("LOGISTIC_REGRESSION"), rc.l2_weight(1.0), nc)
        o = build_optimizer(OptimizerConfig(opt, 200, 1e-10), None, rc, 1.0, track_state=False)
        w, f, _ = optimize_feature_sharded(o, obj, gd, normalization=nc)
        np.save(f"{out}/fsdp_{opt}_{reg}_{norm}_r{rank}.npy", w.numpy())
    from photon_ml_amd.estimators.game_estimator import train_generalized_linear_model
    m = train_generalized_linear_model(local, "LOGISTIC_REGRESSION", "TRON", RegularizationContext("L2"), [1.0],
                                       max_iterations=100, tolerance=1e-10, compute_variance=True, device="cpu",
                                       feature_sharded=True)[0][1]
    np.save(f"{out}/fsdp_api_r{rank}.npy", np.stack([m.coefficients.means.numpy(), m.coefficients.variances.numpy()]))
    import torch.distributed as dist
    dist.destroy_process_group()


def a2a_worker(rank, world, port, out):
    """RowRouter._a2a_device in several rounds (tiny A2A_MAX_BYTES) == one all-to-all, for uneven segments
    (including empty ones) and a 2-d payload."""
    _init(rank, world, port)
    import torch.distributed as dist
    from photon_ml_amd.parallel import sharding
    from photon_ml_amd.parallel.sharding import RowRouter
    rng = np.random.default_rng(100 + rank)
    sc = [int(v) for v in rng.integers(0, 40, world)]
    sc[(rank + 1) % world] = 0                                   # an empty segment
    rc_t = torch.tensor(sc, dtype=torch.int64)
    allc = [torch.zeros(world, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(allc, rc_t)
    rc = [int(allc[q][rank]) for q in range(world)]
    send = torch.arange(sum(sc) * 3, dtype=torch.float64).reshape(-1, 3) + 1000 * rank
    ref = torch.empty((sum(rc), 3), dtype=torch.float64)
    dist.all_to_all_single(ref, send, rc, sc)
    router = RowRouter.__new__(RowRouter)
    router.group = None
    for limit in (8, 50, 1 << 30):
        sharding.A2A_MAX_BYTES = limit
        got = router._a2a_device(send, sc, rc, (3,))
        assert torch.equal(got, ref), (rank, limit)
    np.save(f"{out}/a2a_r{rank}.npy", np.array([1]))
    dist.destroy_process_group()


def sparse_re_data():
    """GAME data with a third random-effect type of only TWO entities (``regionId``): at world 4 / 8 most ranks own
    no entity of it (empty local problems, empty routing sends, empty model parts)."""
    from photon_ml_amd.data.game_data import generate_game_data
    data, _ = generate_game_data(n_rows=3000, n_users=40, n_items=25, seed=31, task="LOGISTIC_REGRESSION")
    data.id_tags["regionId"] = np.array([f"r{int(i[1:]) % 2}" if isinstance(i, str) else int(i) % 2
                                         for i in data.id_tags["itemId"]], dtype=object)
    data.shards["region"] = data.shards["item"]
    return data


def sparse_re_estimator(device="cpu"):
    from photon_ml_amd.data.random_effect import FixedEffectDataConfiguration, RandomEffectDataConfiguration
    from photon_ml_amd.estimators.game_estimator import GameEstimator
    return (GameEstimator(device=device).set_training_task("LOGISTIC_REGRESSION")
            .set_coordinate_data_configurations({"global": FixedEffectDataConfiguration("global"),
                                                 "per-user": RandomEffectDataConfiguration("userId", "user"),
                                                 "per-region": RandomEffectDataConfiguration("regionId", "region")})
            .set_coordinate_update_sequence(["global", "per-user", "per-region"])
            .set_coordinate_descent_iterations(2)
            .set_validation_evaluators(["AUC", "AUC:regionId", "LOGISTIC_LOSS"]))


def sparse_re_worker(rank, world, port, out):
    """A random-effect type with fewer entities than ranks: ranks owning none of them still run the coordinate
    (zero local entities), the evaluators and the per-rank model parts; the result equals the single process."""
    _init(rank, world, port)
    from photon_ml_amd.io.index_map import DefaultIndexMap
    from photon_ml_amd.io.model_io import save_game_model
    from photon_ml_amd.optimization.config import (GLMOptimizationConfiguration, OptimizerConfig,
                                                   RegularizationContext)
    data = sparse_re_data()
    tr, va = data.subset(np.arange(2400)), data.subset(np.arange(2400, 3000))
    tr_l = tr.subset(np.arange(rank, tr.n_rows, world))
    va_l = va.subset(np.arange(rank, va.n_rows, world))
    cfg = GLMOptimizationConfiguration(OptimizerConfig("TRON", 50, 1e-10), RegularizationContext("L2"), 1.0)
    est = sparse_re_estimator()
    res = est.fit(tr_l, va_l, [{"global": cfg, "per-user": cfg, "per-region": cfg}])[0]
    owned = len(est.coordinates["per-region"].dataset.entity_ids) if hasattr(
        est.coordinates["per-region"], "dataset") else -1
    np.save(f"{out}/sparse_owned_r{rank}.npy", np.array([owned]))
    np.save(f"{out}/sparse_fe_r{rank}.npy", res.model.get("global").glm.coefficients.means.numpy())
    np.save(f"{out}/sparse_eval_r{rank}.npy", np.array([v for _, v in res.evaluations]))
    maps = {s: DefaultIndexMap.from_keys([f"f{j}\u0001t" for j in range(data.shards[s].shape[1])])
            for s in data.shards}
    save_game_model(res.model, f"{out}/model", maps, opt_configs=res.config)
    import torch.distributed as dist
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    fn = {"glm": glm_worker, "game": game_worker, "sharding": sharding_worker, "fsdp": fsdp_worker,
          "placed": placed_worker, "sparse_re": sparse_re_worker, "a2a": a2a_worker}[sys.argv[1]]
    fn(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5])
