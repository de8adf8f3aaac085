"""The multi-GPU form of the C ABI (dpg_ctx_create_multi): one process drives the
devices, edges are sharded over them, every Gauss-Newton iteration all-reduces the packed system
with RCCL (ncclAllReduce on the devices' streams).  The GPU box has one card, so these tests run
the multi-GPU context at n_gpus = 1 -- the sharded code paths, the RCCL communicator and its
all-reduce with one rank -- and require results byte-identical to the single-device context.
(The N > 1 collectives are the driver's 8-GPU run; tests/test_dist_gpu.py and test_dist_cpu.py
cover the sharding arithmetic with more ranks.)"""
import numpy as np
import pytest


@pytest.mark.gpu
def test_multi_ctx_one_gpu_equals_single_device(workload):
    from dpgslam import _abi, api
    w = workload("config3")
    p = _abi.default_icp_params()
    single = api.Context(0)
    multi = api.Context(0, n_gpus=1)
    assert multi.n_gpus == 1 and single.n_gpus == 1
    out = []
    for ctx in (single, multi):
        ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
        res, hess = ctx.icp_batch(w.edges, w.est, p, compute_cov=True)
        F = w.factors_with_icp(res, p)
        X, st = ctx.optimize_graph(w.est.astype(np.float64), F)
        passes = np.zeros(w.V, np.int32)
        Xr, sr = ctx.reoptimize(passes, w.est, w.odom)
        out.append((res.tobytes(), np.asarray(hess).tobytes(), X.tobytes(), st.iterations, Xr.tobytes(),
                    sr.n_loop_closures, sr.gn.iterations))
    a, b = out
    assert a[0] == b[0], "ICP results differ"
    assert a[1] == b[1], "covariance blocks differ"
    assert a[2] == b[2] and a[3] == b[3], "optimize_graph differs"
    assert a[4] == b[4] and a[5] == b[5] and a[6] == b[6], "reoptimize differs"
    # the per-device step API and the incremental graph want a single-device context
    with pytest.raises(_abi.DpgError):
        api.IncGraph(multi)
    multi.close()
    single.close()
