"""Single-GPU RCCL worker for ``test_rccl_gpu.py``.

``forced`` mode runs with ``WORLD_SIZE=1 PML_FORCE_DIST=1`` and the ``nccl`` (= RCCL) backend, so every
multi-rank code path goes through real RCCL collectives on the device: the bucketed asynchronous gradient
all-reduce overlapped with the transpose kernels (``DistributedGLMData._packed_overlap`` and the accepted-step
reduction of the margin-space line search), the Hessian-vector reduction of TRON, feature-sharded optimizer state
(all-gather / reduce-scatter) and the entity-sharded GAME coordinate (device all-to-all row routing). ``plain``
mode computes the same things without a process group. The test compares the two.
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(mode, out):
    from photon_ml_amd.parallel.dist import DistributedGLMData, init_distributed, is_dist
    init_distributed("nccl" if mode == "forced" else None)
    assert is_dist() == (mode == "forced")
    import torch.distributed as dist
    if mode == "forced":
        assert dist.get_backend() == "nccl"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)

    from photon_ml_amd.data.synthetic import generate_device_shard
    from photon_ml_amd.function.losses import LOGISTIC, POISSON
    from photon_ml_amd.function.objective import GLMObjective
    from photon_ml_amd.optimization.lbfgs import LBFGS
    from photon_ml_amd.optimization.tron import TRON

    # ---- data-parallel GLM: L-BFGS (gradient + line-search reductions) and TRON (Hessian-vector reductions)
    for name, task, loss, mk in (("lbfgs", "LOGISTIC_REGRESSION", LOGISTIC, lambda: LBFGS(tolerance=0.0,
                                                                                          max_iterations=10 ** 9)),
                                 ("tron", "POISSON_REGRESSION", POISSON, lambda: TRON(tolerance=0.0,
                                                                                      max_iterations=10 ** 9))):
        data, _ = generate_device_shard(300_000, 20_000, 30, dev, "bf16", seed=11, chunk_rows=1 << 17, task=task)
        gdata = data
        if is_dist():
            gdata = DistributedGLMData(data)
            assert gdata.overlap, "bucketed overlapped all-reduce must be on (one feature order)"
        obj = GLMObjective(loss, l2_weight=1.0)
        opt = mk()
        opt.start(obj, gdata, torch.zeros(data.dim, dtype=torch.float64, device=dev), skip_zero_tolerance_pass=True)
        for _ in range(4):
            st = opt.step(obj, gdata)
        torch.cuda.synchronize()
        np.save(f"{out}/{mode}_{name}_w.npy", st.coefficients.cpu().numpy())
        np.save(f"{out}/{mode}_{name}_f.npy", np.array([st.loss]))
        del data, gdata

    # ---- feature-sharded optimizer state (all-gather w / reduce-scatter g over RCCL)
    if is_dist():
        from photon_ml_amd.optimization.vector_space import ShardedSpace, active_space
        from photon_ml_amd.parallel.feature_sharding import FeatureShardLayout, FeatureShardedObjective
        data, _ = generate_device_shard(200_000, 10_000, 20, dev, "bf16", seed=12, chunk_rows=1 << 17)
        layout = FeatureShardLayout.current(data.dim)
        obj = FeatureShardedObjective(GLMObjective(LOGISTIC, l2_weight=1.0), layout)
        opt = LBFGS(tolerance=0.0, max_iterations=10 ** 9)
        with active_space(ShardedSpace()):
            opt.start(obj, data, layout.slice(torch.zeros(data.dim, dtype=torch.float64, device=dev)).clone(),
                      skip_zero_tolerance_pass=True)
            for _ in range(4):
                st = opt.step(obj, data)
        torch.cuda.synchronize()
        np.save(f"{out}/{mode}_fsdp_w.npy", st.coefficients.cpu().numpy())
        del data
    else:
        data, _ = generate_device_shard(200_000, 10_000, 20, dev, "bf16", seed=12, chunk_rows=1 << 17)
        opt = LBFGS(tolerance=0.0, max_iterations=10 ** 9)
        obj = GLMObjective(LOGISTIC, l2_weight=1.0)
        opt.start(obj, data, torch.zeros(data.dim, dtype=torch.float64, device=dev), skip_zero_tolerance_pass=True)
        for _ in range(4):
            st = opt.step(obj, data)
        torch.cuda.synchronize()
        np.save(f"{out}/{mode}_fsdp_w.npy", st.coefficients.cpu().numpy())
        del data

    # ---- GAME: fixed effect + entity-sharded random effects (ShardedRandomEffectCoordinate under a group)
    from photon_ml_amd.data.game_data import generate_game_data
    from photon_ml_amd.data.random_effect import FixedEffectDataConfiguration, RandomEffectDataConfiguration
    from photon_ml_amd.estimators.game_estimator import GameEstimator
    from photon_ml_amd.optimization.config import (GLMOptimizationConfiguration, OptimizerConfig,
                                                   RegularizationContext)
    gd, _ = generate_game_data(n_rows=4000, n_users=40, n_items=25, seed=21, task="LOGISTIC_REGRESSION")
    cfg = GLMOptimizationConfiguration(OptimizerConfig("TRON", 100, 1e-10), RegularizationContext("L2"), 1.0)
    est = (GameEstimator(device="cuda", precision="f64").set_training_task("LOGISTIC_REGRESSION")
           .set_coordinate_data_configurations({"global": FixedEffectDataConfiguration("global"),
                                                "per-user": RandomEffectDataConfiguration("userId", "user"),
                                                "per-item": RandomEffectDataConfiguration("itemId", "item")})
           .set_coordinate_update_sequence(["global", "per-user", "per-item"])
           .set_coordinate_descent_iterations(2)
           .set_validation_evaluators(["AUC", "LOGISTIC_LOSS"]))
    res = est.fit(gd, gd, [{"global": cfg, "per-user": cfg, "per-item": cfg}])[0]
    np.save(f"{out}/{mode}_game_fe.npy", res.model.get("global").glm.coefficients.means.cpu().numpy())
    np.save(f"{out}/{mode}_game_eval.npy", np.array([v for _, v in res.evaluations]))
    for cid in ("per-user", "per-item"):
        m = res.model.get(cid)
        order = np.argsort(np.asarray(m.keys).astype(str))
        np.save(f"{out}/{mode}_game_{cid}.npy", np.asarray(m.values)[order])
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    print(f"{mode} ok", flush=True)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
