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

from multi_common import compare, perr, run_all, run_step


@pytest.fixture(scope="module")
def single_run(workload):
    from dpgslam import _abi, api
    w = workload("config3")
    p = _abi.default_icp_params()
    with api.Context(0) as c:
        return run_all(c, w, p)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [2, 3])
def test_virtual_devices_equal_single_device(workload, single_run, k):
    from dpgslam import _abi, api
    w = workload("config3")
    p = _abi.default_icp_params()
    with api.Context(0, virtual=k) as c:
        assert c.n_gpus == k and c.n_ranks == k
        out = run_all(c, w, p)
    compare(out, single_run)


@pytest.fixture(scope="module")
def single_step4(workload):
    from dpgslam import _abi, api
    w = workload("config4")
    p = _abi.default_icp_params()
    with api.Context(0) as c:
        c.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
        return run_step(c, w, p)


@pytest.mark.gpu
@pytest.mark.parametrize("schedule", ["caller", "measured"])
def test_virtual8_config4_equals_single_device(workload, single_step4, schedule):
    """The target world size at the headline size (BASELINE config 4, 8 GPUs): k = 8 virtual
    devices run the bench step twice (the second run planned from measured costs under 'measured')
    -- every ICP result and covariance block byte-identical to one device, the same GN iterations
    and factorizations, poses within 1e-9."""
    from dpgslam import _abi, api
    w = workload("config4")
    p = _abi.default_icp_params()
    with api.Context(0, virtual=8) as c:
        assert c.n_gpus == 8 and c.n_ranks == 8
        c.set_icp_schedule(schedule)
        c.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
        out = run_step(c, w, p)
    for k in (0, 1):
        assert out[f"rs{k}"] == single_step4[f"rs{k}"], f"ICP results of run {k} differ"
        assert out[f"hs{k}"] == single_step4[f"hs{k}"], f"covariance blocks of run {k} differ"
        assert out[f"its{k}"] == single_step4[f"its{k}"] and out[f"nfs{k}"] == single_step4[f"nfs{k}"]
        assert perr(out[f"Xs{k}"], single_step4[f"Xs{k}"]) < 1e-9


@pytest.mark.gpu
def test_multi_ctx_one_gpu_equals_single_device(workload, single_run):
    """dpg_ctx_create_multi(1): the RCCL all-reduce with one rank -- byte-identical everything."""
    from dpgslam import _abi, api
    w = workload("config3")
    p = _abi.default_icp_params()
    with api.Context(0, n_gpus=1) as c:
        assert c.n_gpus == 1 and c.n_ranks == 1
        out = run_all(c, w, p)
        # the per-iteration step API and the incremental graph want a single-device context
        with pytest.raises(_abi.DpgError):
            api.IncGraph(c)
        with pytest.raises(_abi.DpgError):
            c.gn_assemble()
    compare(out, single_run, exact_poses=True)


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
        out = run_all(c, w, p)
    compare(out, single_run, exact_poses=True)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["config3", "config4"])
def test_rank_form_two_ranks_on_one_card(cfg):
    """dpg_ctx_create_rank_ops at world = 2: two processes share the card, libdpg's rank form with
    gloo as its collective (tools/rank_check.py) -- the cost all-reduce of the LPT plan, the results'
    all-gather, factor ownership by global rank and the packed system's all-reduce per iteration all
    run for real.  Both schedules; each rank's results byte-identical to a single-device context, the
    same iteration / factorization counts, poses within 1e-9, and the ranks issued the same
    collectives."""
    import os
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([root, os.path.join(root, "dpg-slam_amd"),
                                                         os.path.join(root, "tests")]))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port),
                        os.path.join(root, "tools", "rank_check.py"), cfg],
                       capture_output=True, text=True, timeout=240, env=env)
    print(r.stdout[-3000:])
    assert r.returncode == 0 and r.stdout.count("rank check ok") == 2, (r.stdout + r.stderr)[-4000:]


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
