"""The multi-device forms of the C ABI: dpg_ctx_create_multi (one process, RCCL
between its devices), dpg_ctx_create_rank (one process per GPU) and dpg_ctx_create_virtual (k
contexts on one device sharing a stream, the all-reduce a device-side sum).  The GPU box has one
card, so the sharded code paths -- edge assignment, per-device staging, the gather of results in
the caller's order, the factor ownership and the device-side ICP-to-factor scatter, the all-reduce
between assembly and decision, every device's own stop / chord decisions -- run here on k = 2 and
3 VIRTUAL devices, and the RCCL form at n_gpus = 1.  Bar: ICP results byte-identical to the
single-device context (both dispatch schedules), poses within 1e-9 and the same iteration /
factorization counts for dpg_optimize_graph, dpg_reoptimize and the step form the bench runs."""
import numpy as np
import pytest

from conftest import angle_wrap


def _perr(A, B):
    return float(np.abs(np.concatenate([A[:, :2] - B[:, :2], angle_wrap(A[:, 2:] - B[:, 2:])], 1)).max())


def _run_all(ctx, w, p):
    """ICP batch (+ covariance) twice (the second run re-plans from the first run's costs), the
    graph solve, the bench's step form, and a sweep."""
    from dpgslam import _abi
    ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
    res1, hess1 = ctx.icp_batch(w.edges, w.est, p, compute_cov=True)
    ctx.icp_run(compute_cov=True)           # again: the measured schedule now (LPT + longest first)
    res2, hess2 = ctx.icp_fetch(with_hessian=True)
    F = w.factors_with_icp(res1, p)
    X, st = ctx.optimize_graph(w.est.astype(np.float64), F)
    # the bench's step: the staged batch's results become factors on the device(s) that aligned them
    ctx.icp_prepare(w.edges, w.est, p)
    ctx.icp_run(compute_cov=False)
    gp = _abi.default_gn_params()
    ctx.gn_setup(w.V, w.factors_placeholder(), params=gp)
    ctx.gn_take_icp(w.icp_factor_first, w.E, w.n_successive, p)
    ctx.gn_set_poses(w.est.astype(np.float64))
    sst, Xs = ctx.gn_run(w.V)
    nfs = ctx.gn_factorizations()
    passes = np.zeros(w.V, np.int32)
    passes[w.V // 2:] = 1
    Xr, sr = ctx.reoptimize(passes, w.est, w.odom)
    rr, _ = ctx.icp_fetch(with_hessian=False)
    return dict(res1=res1.tobytes(), hess1=np.asarray(hess1).tobytes(), res2=res2.tobytes(),
                hess2=np.asarray(hess2).tobytes(), X=X, it=st.iterations, Xs=Xs, its=sst["iterations"], nfs=nfs,
                err_s=sst["final_error"], Xr=Xr, itr=sr.gn.iterations, nlc=sr.n_loop_closures, rr=rr.tobytes())


@pytest.fixture(scope="module")
def single_run(workload):
    from dpgslam import _abi, api
    w = workload("config3")
    p = _abi.default_icp_params()
    with api.Context(0) as c:
        return _run_all(c, w, p)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [2, 3])
def test_virtual_devices_equal_single_device(workload, single_run, k):
    from dpgslam import _abi, api
    w = workload("config3")
    p = _abi.default_icp_params()
    with api.Context(0, virtual=k) as c:
        assert c.n_gpus == k and c.n_ranks == k
        out = _run_all(c, w, p)
    a = single_run
    for key in ("res1", "hess1", "res2", "hess2", "rr"):
        assert out[key] == a[key], f"{key} differs from the single-device context"
    assert out["it"] == a["it"] and _perr(out["X"], a["X"]) < 1e-9
    assert out["its"] == a["its"] and out["nfs"] == a["nfs"] and _perr(out["Xs"], a["Xs"]) < 1e-9
    assert abs(out["err_s"] - a["err_s"]) <= 1e-9 * max(1.0, abs(a["err_s"]))
    assert out["itr"] == a["itr"] and out["nlc"] == a["nlc"] and _perr(out["Xr"], a["Xr"]) < 1e-9


@pytest.mark.gpu
def test_multi_ctx_one_gpu_equals_single_device(workload, single_run):
    """dpg_ctx_create_multi(1): the RCCL all-reduce with one rank -- byte-identical everything."""
    from dpgslam import _abi, api
    w = workload("config3")
    p = _abi.default_icp_params()
    with api.Context(0, n_gpus=1) as c:
        assert c.n_gpus == 1 and c.n_ranks == 1
        out = _run_all(c, w, p)
        # the per-iteration step API and the incremental graph want a single-device context
        with pytest.raises(_abi.DpgError):
            api.IncGraph(c)
        with pytest.raises(_abi.DpgError):
            c.gn_assemble()
    a = single_run
    for key in ("res1", "hess1", "res2", "hess2", "rr"):
        assert out[key] == a[key], key
    assert out["X"].tobytes() == a["X"].tobytes() and out["it"] == a["it"]
    assert out["Xs"].tobytes() == a["Xs"].tobytes() and out["its"] == a["its"] and out["nfs"] == a["nfs"]
    assert out["Xr"].tobytes() == a["Xr"].tobytes() and out["itr"] == a["itr"] and out["nlc"] == a["nlc"]


@pytest.mark.gpu
def test_rank_form_one_rank_equals_single_device(workload, single_run):
    """dpg_ctx_create_rank with world 1 (the torchrun form's communicator from a unique id)."""
    from dpgslam import _abi, api
    w = workload("config3")
    p = _abi.default_icp_params()
    nid = api.nccl_unique_id()
    assert len(nid) == api.NCCL_ID_BYTES
    with api.Context(0, rank=(nid, 0, 1)) as c:
        assert c.n_ranks == 1 and c.rank == 0
        out = _run_all(c, w, p)
    a = single_run
    for key in ("res1", "hess1", "res2", "rr"):
        assert out[key] == a[key], key
    assert out["Xs"].tobytes() == a["Xs"].tobytes() and out["its"] == a["its"]


@pytest.mark.gpu
def test_schedules_and_shard_sizes(workload):
    """Both dispatch schedules give the same bytes; the measured one balances the shards by cost
    (LPT) -- every virtual device gets a share, and a batch whose pairs were all aligned before is
    planned from the costs at once."""
    from dpgslam import _abi, api
    w = workload("config2")
    p = _abi.default_icp_params()
    outs = []
    for sched in ("caller", "measured"):
        with api.Context(0, virtual=3) as c:
            c.set_icp_schedule(sched)
            c.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
            r1, _ = c.icp_batch(w.edges, w.est, p, compute_cov=False)
            r2, _ = c.icp_batch(w.edges, w.est, p, compute_cov=False)   # pairs known: planned at prepare
            outs += [r1.tobytes(), r2.tobytes()]
    assert all(o == outs[0] for o in outs)
    with api.Context(0, virtual=2) as c:
        c.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
        c.icp_prepare(w.edges, w.est, p)
        c.icp_run(compute_cov=False)
        with pytest.raises(_abi.DpgError):   # a multi-device context takes the whole batch
            c.gn_setup(w.V, w.factors_placeholder())
            c.gn_take_icp(w.icp_factor_first, w.E - 1, w.n_successive, p)


@pytest.mark.gpu
def test_bench_refuses_more_gpus_than_visible():
    """bench.py --gpus N without a launcher opens N devices in one process; with fewer visible it
    must fail loudly (exit code 2), not measure one GPU."""
    import os
    import subprocess
    import sys
    import torch
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    n = torch.cuda.device_count()
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(n + 1), "--steps", "1",
                        "--warmup", "0", "--no-cpu-baseline"], capture_output=True, text=True, timeout=180,
                       env={k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")})
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "visible" in r.stderr
