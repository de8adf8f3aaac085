"""GPU tests of the pose-graph solver itself: the one-launch DAG Cholesky against
the level-scheduled one, a known-answer mesh graph whose elimination tree has large fronts (the
multi-workgroup team path), and the asynchronous GN loop against dpg_optimize_graph."""
import numpy as np
import pytest

from graphs import consistent_mesh_graph, pose_diff

pytestmark = pytest.mark.gpu


def _optimize(ctx, X0, F, levels=False, solver=None, **kw):
    """dpg_optimize_graph with solver options (dpg_ctx_set_solver_options, taken when the graph is
    set up), the defaults restored afterwards."""
    from dpgslam import _abi
    gp = _abi.default_gn_params()
    for k, v in kw.items():
        setattr(gp, k, v)
    opts = dict(solver or {})
    if levels:
        opts["fused"] = 0
    ctx.set_solver_options(**opts)
    try:
        return ctx.optimize_graph(X0, F, gp)
    finally:
        ctx.set_solver_options()


def test_mesh_graph_known_answer(ctx):
    """Exactly consistent measurements: GN reaches the true poses; the fused DAG factorization and
    the level-scheduled one agree."""
    X0, F, X = consistent_mesh_graph(V=3000, k=6, seed=11)
    Xf, sf = _optimize(ctx, X0, F)
    assert np.abs(pose_diff(Xf, X)).max() < 1e-8, np.abs(pose_diff(Xf, X)).max()
    Xl, sl = _optimize(ctx, X0, F, levels=True)
    assert np.abs(pose_diff(Xl, X)).max() < 1e-8
    assert sf.iterations == sl.iterations
    assert np.abs(pose_diff(Xf, Xl)).max() < 1e-10


@pytest.mark.parametrize("name", ["config3", "config4"])
def test_fused_and_level_cholesky_agree(ctx, workload, name):
    from oracle import oracle as O
    from dpgslam import _abi
    w = workload(name)
    p = _abi.default_icp_params()
    ctx.upload_scans(w.pts, w.offsets, 5)
    res, _ = ctx.icp_batch(w.edges, w.est, p, compute_cov=False)
    F = w.factors_with_icp(res, p)
    X0 = w.est.astype(np.float64)
    Xf, sf = _optimize(ctx, X0, F)
    Xl, sl = _optimize(ctx, X0, F, levels=True)
    assert sf.iterations == sl.iterations
    assert np.abs(pose_diff(Xf, Xl)).max() < 1e-9
    if name == "config3":
        Xo, _ = O.optimize_graph(X0, F)
        assert np.abs(pose_diff(Xf, Xo)).max() < 1e-6


def test_async_gn_loop_matches_optimize_graph(ctx, workload):
    """dpgslam.dist.gn_loop on the device backend (enqueue-only solve/retract, one fetch per
    iteration) performs exactly dpg_optimize_graph's operations: identical poses and iterations."""
    import torch
    from dpgslam import _abi
    from dpgslam import dist as D
    w = workload("config3")
    p = _abi.default_icp_params()
    ctx.upload_scans(w.pts, w.offsets, 5)
    res, _ = ctx.icp_batch(w.edges, w.est, p, compute_cov=False)
    F = w.factors_with_icp(res, p)
    X0 = w.est.astype(np.float64)
    Xc, sc = ctx.optimize_graph(X0, F)
    dev = torch.device("cuda", 0)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    n = ctx.gn_setup(w.V, F)
    ctx.gn_set_poses(X0)
    st = D.gn_loop(D.DeviceBackend(ctx, n, n - 2, dev), lambda hb: None, _abi.default_gn_params())
    Xa = ctx.gn_get_poses(w.V)
    assert st["iterations"] == sc.iterations
    np.testing.assert_array_equal(Xa, Xc)
    # dpg_gn_run: the same loop natively, from the same staged graph and poses
    ctx.gn_set_poses(X0)
    sn, Xn = ctx.gn_run(w.V)
    assert sn["iterations"] == sc.iterations
    assert sn["final_error"] == st["final_error"]
    np.testing.assert_array_equal(Xn, Xc)


@pytest.mark.parametrize("name", ["config3", "config4"])
def test_orders_agree(ctx, workload, name):
    """The nested-dissection order (default: the better of two separator rules), round 2's rule
    alone and plain minimum degree (dpg_solver_options.order) factor the same system: the GN
    solutions agree to rounding, and against the oracle on config 3."""
    from oracle import oracle as O
    from dpgslam import _abi
    w = workload(name)
    p = _abi.default_icp_params()
    ctx.upload_scans(w.pts, w.offsets, 5)
    res, _ = ctx.icp_batch(w.edges, w.est, p, compute_cov=False)
    F = w.factors_with_icp(res, p)
    X0 = w.est.astype(np.float64)
    Xn, sn = _optimize(ctx, X0, F)
    Xm, sm = _optimize(ctx, X0, F, solver={"order": "md"})
    Xr, sr = _optimize(ctx, X0, F, solver={"order": "nd"})
    assert np.abs(pose_diff(Xn, Xm)).max() < 1e-9
    assert np.abs(pose_diff(Xn, Xr)).max() < 1e-9
    if name == "config3":
        Xo, _ = O.optimize_graph(X0, F)
        assert np.abs(pose_diff(Xn, Xo)).max() < 1e-6


@pytest.mark.parametrize("opts", [{"solve_stage": 0}, {"solve_stage": 15000}, {"solve_maxseg": 0}, {"solve_maxseg": 1},
                                  {"merge_single": 1}, {"solve_dinv": 1}, {"solve_inv_cols": 48}])
def test_solve_paths_agree(ctx, workload, opts):
    """The triangular solves' code paths give the same GN solution on config 4 (chord steps and
    fresh factorizations): no LDS staging, staging of whole fronts up to 15 000 doubles, the
    backward solve with every front waiting for its parent (no row segments) or with segments only
    where there is one, the single-child supernode rule, the inverted diagonal blocks, and the
    large fronts' L11^-1 computed beside the pipelined loop's solves -- against the defaults
    (dpg_solver_options)."""
    from dpgslam import _abi
    w = workload("config4")
    p = _abi.default_icp_params()
    ctx.upload_scans(w.pts, w.offsets, 5)
    res, _ = ctx.icp_batch(w.edges, w.est, p, compute_cov=False)
    F = w.factors_with_icp(res, p)
    X0 = w.est.astype(np.float64)
    Xd, sd = _optimize(ctx, X0, F)
    Xe, se = _optimize(ctx, X0, F, solver=opts)
    assert se.iterations == sd.iterations
    assert np.abs(pose_diff(Xe, Xd)).max() < 1e-9


def test_zero_initial_error_runs_no_iteration(ctx, workload):
    """The pipelined loop takes the initial error on the device (no host round trip before the first
    iteration): a graph already at its optimum runs no iteration, and the reported initial error
    equals the host-decided loop's (the PCG solver reads it back first) on a real graph."""
    from dpgslam import _abi, api
    F = np.concatenate([api.prior_factor(0), api.between_factor(0, 1, (1.0, 0.0, 0.0), sigmas=(0.1, 0.1, 0.05))])
    X0 = np.array([[0.0, 0.0, 0.0], [1.0, 0.0, 0.0]])
    for solver in (_abi.DPG_SOLVER_CHOLESKY, _abi.DPG_SOLVER_PCG):
        X, st = _optimize(ctx, X0, F, linear_solver=solver)
        assert st.iterations == 0 and st.initial_error == 0.0 and st.final_error == 0.0, (solver, st.iterations)
        assert np.array_equal(X, X0)
    w = workload("config3")
    p = _abi.default_icp_params()
    ctx.upload_scans(w.pts, w.offsets, 5)
    res, _ = ctx.icp_batch(w.edges, w.est, p, compute_cov=False)
    Fw = w.factors_with_icp(res, p)
    X0w = w.est.astype(np.float64)
    _, sc = _optimize(ctx, X0w, Fw)
    _, sp = _optimize(ctx, X0w, Fw, linear_solver=_abi.DPG_SOLVER_PCG)
    assert sc.initial_error == sp.initial_error > 0.0
