"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle.

Bar (DESIGN.md "Parity"): correspondence indices, transforms, iteration counts, convergence flags
and MSE BIT-EXACT; covariance block within 1e-12 relative; poses within 1e-6 (max abs x, y, theta).
"""
import numpy as np
import pytest

from graphs import gtsam_test_graph, pose_diff

pytestmark = pytest.mark.gpu


def _oracle():
    from oracle import oracle as O
    return O


def _params(ratio=5):
    from dpgslam import _abi
    p = _abi.default_icp_params()
    p.downsample_icp_points_ratio = ratio
    return p


def _assert_results_equal(gpu, ref, what=""):
    for k in ("T", "z", "converged", "iterations", "n_corr", "status", "fitness"):
        g, r = np.asarray(gpu[k]), np.asarray(ref[k])
        bad = np.nonzero(~np.all((g == r).reshape(len(g), -1), axis=1))[0] if g.ndim > 0 else []
        assert len(bad) == 0, f"{what}: field {k} differs on {len(bad)} edges, first {bad[:5]}: {g[bad[:3]]} vs {r[bad[:3]]}"


@pytest.mark.parametrize("ratio", [5, 1])
def test_config1_single_alignment_bit_exact(ctx, workload, ratio):
    """config 1: two 360-beam scans, one runIcp; per-iteration correspondences bit-exact."""
    from dpgslam import _abi, api
    O = _oracle()
    w = workload("config1")
    p = _params(ratio)
    src_ds, tgt_ds = api.downsample(w.cloud(1), ratio), api.downsample(w.cloud(0), ratio)
    guess = api.icp_guess(w.est[1], w.est[0])
    ref, ref_tr = O.icp_align(src_ds, tgt_ds, guess, p, O.NN_BRUTE, trace_iters=64)
    ok, z, cov, res, hess = ctx.run_icp(w.node(0), w.node(1), p, with_hessian=True)
    r = np.frombuffer(bytes(res), _abi.RESULT_DTYPE)
    rr = np.frombuffer(bytes(ref), _abi.RESULT_DTYPE)
    _assert_results_equal(r, rr, "config1")
    assert ok == bool(ref.converged)
    np.testing.assert_array_equal(cov, np.diag(np.array([0.5, 0.5, 0.3], np.float32).astype(np.float64)))
    _, ref_h = O.icp_cov(w.cloud(1), w.cloud(0), np.array(ref.T))
    np.testing.assert_allclose(hess, ref_h, rtol=1e-12, atol=1e-9)
    # per-iteration correspondences through the batch path
    ctx.upload_scans(w.pts, w.offsets, ratio)
    ctx.icp_batch(w.edges, w.est, p, compute_cov=True, trace_iters=64)
    tr = ctx.icp_fetch_trace(64)[0]
    n = ref.iterations
    np.testing.assert_array_equal(tr[:n, :len(src_ds)], ref_tr[:n])


@pytest.mark.parametrize("variant", ["angular", "kdtree", "grid"])
def test_icp_batch_config2_bit_exact(ctx, workload, variant):
    """config 2: all 499 successive edges of the 500-node chain, full ICP outcome bit-exact and the
    first 40 iterations' correspondence indices bit-exact on 16 edges (every NN variant)."""
    O = _oracle()
    w = workload("config2")
    p = _params()
    ctx.set_icp_variant(variant)
    ctx.upload_scans(w.pts, w.offsets, 5)
    res, hess = ctx.icp_batch(w.edges, w.est, p, compute_cov=True, trace_iters=40)
    ref, ref_h = O.icp_batch(w.pts, w.offsets, w.edges, w.est, p, O.NN_GRID, threads=16)
    _assert_results_equal(res, ref, "config2")
    np.testing.assert_allclose(hess, ref_h, rtol=1e-12, atol=1e-8)
    tr = ctx.icp_fetch_trace(40)
    from dpgslam import api
    for e in range(0, w.E, max(1, w.E // 16)):
        t, s = w.edges[e]
        sd, td = api.downsample(w.cloud(s), 5), api.downsample(w.cloud(t), 5)
        r1, rt = O.icp_align(sd, td, api.icp_guess(w.est[s], w.est[t]), p, O.NN_BRUTE, trace_iters=40)
        n = min(r1.iterations, 40)
        np.testing.assert_array_equal(tr[e, :n, :len(sd)], rt[:n], err_msg=f"edge {e}")
    ctx.set_icp_variant("angular")


def test_icp_cov_calculate_constant(ctx, workload):
    """calculate_ICP_COV returns diag(var_x, var_y, var_theta) exactly (cov :572-575)."""
    from dpgslam import api
    O = _oracle()
    w = workload("config1")
    T = np.eye(4, dtype=np.float32)
    T[0, 0] = T[1, 1] = np.float32(np.cos(0.3))
    T[1, 0] = np.float32(np.sin(0.3))
    T[0, 1] = -T[1, 0]
    T[0, 3], T[1, 3] = 0.4, -0.2
    cov, hess = api.calculate_ICP_COV(w.cloud(1), w.cloud(0), T, 0.5, 0.5, 0.3, ctx=ctx)
    assert cov.tobytes() == np.diag([np.float64(np.float32(0.5)), np.float64(np.float32(0.5)),
                                     np.float64(np.float32(0.3))]).tobytes()
    T6 = np.array([T[0, 0], T[0, 1], T[0, 3], T[1, 0], T[1, 1], T[1, 3]], np.float32)
    _, ref = O.icp_cov(w.cloud(1), w.cloud(0), T6)
    np.testing.assert_allclose(hess, ref, rtol=1e-12, atol=1e-9)
    # unequal cloud sizes: the block sums over min(n_data, n_model)
    cov2, hess2 = api.calculate_ICP_COV(w.cloud(1)[:100], w.cloud(0), T, ctx=ctx)
    _, ref2 = O.icp_cov(w.cloud(1)[:100], w.cloud(0), T6)
    np.testing.assert_allclose(hess2, ref2, rtol=1e-12, atol=1e-9)
    assert hess2[0, 0] == 200.0


def test_gtsam_test_graph_gpu():
    """Known answer from the reference's own gtsam_test (dpg_slam_main.cc:217-282)."""
    from dpgslam import _abi, api
    X0, F, X_opt = gtsam_test_graph()
    with api.Context(0) as c:
        for crit in (0, 1):
            gp = _abi.default_gn_params()
            gp.use_error_criteria = crit
            X, st = c.optimize_graph(X0, F, gp)
            assert np.abs(pose_diff(X, X_opt)).max() < 1e-9, (crit, X)


@pytest.mark.parametrize("solver", [0, 1], ids=["cholesky", "pcg"])
@pytest.mark.parametrize("name", ["config2", "config3"])
def test_gn_matches_oracle(ctx, workload, name, solver):
    """Batch GN on the GPU (supernodal Cholesky, or PCG) vs the oracle's block-sparse Cholesky GN:
    poses within 1e-6."""
    from dpgslam import _abi
    O = _oracle()
    w = workload(name)
    p = _params()
    ctx.upload_scans(w.pts, w.offsets, 5)
    res, _ = ctx.icp_batch(w.edges, w.est, p, compute_cov=False)
    F = w.factors_with_icp(res, p)
    X0 = w.est.astype(np.float64)
    gp = _abi.default_gn_params()
    gp.linear_solver = solver
    Xg, sg = ctx.optimize_graph(X0, F, gp)
    Xo, so = O.optimize_graph(X0, F)
    assert sg.iterations < 100 and so.iterations < 100
    err = np.abs(pose_diff(Xg, Xo)).max()
    assert err < 1e-6, f"{name}: max pose error {err}"
    assert abs(sg.final_error - so.final_error) <= 1e-9 * max(1.0, so.final_error)


def test_gn_device_measurements_match_host(ctx, workload):
    """The device-resident pipeline (ICP results -> factors on device) equals the host-built one."""
    w = workload("config3")
    p = _params()
    ctx.upload_scans(w.pts, w.offsets, 5)
    res, _ = ctx.icp_batch(w.edges, w.est, p, compute_cov=False)
    F_host = w.factors_with_icp(res, p)
    Xh, _ = ctx.optimize_graph(w.est.astype(np.float64), F_host)
    ctx.gn_setup(w.V, w.factors_placeholder())
    ctx.gn_take_icp(w.icp_factor_first, w.E, w.n_successive, p)
    ctx.gn_set_poses(w.est.astype(np.float64))
    for _ in range(100):
        ctx.gn_assemble()
        dinf, _, _ = ctx.gn_solve_retract()
        if dinf < 1e-10:
            break
    Xd = ctx.gn_get_poses(w.V)
    assert np.abs(pose_diff(Xd, Xh)).max() < 1e-6


@pytest.mark.slow
def test_config4_full_size(ctx, workload):
    """config 4 at full size: 20000 ICP edges bit-exact vs the oracle, then GN poses < 1e-6, and the
    size-independent property that the covariance block's (0,0) entry is 2 * min(n_data, n_model)."""
    O = _oracle()
    w = workload("config4")
    p = _params()
    ctx.upload_scans(w.pts, w.offsets, 5)
    res, hess = ctx.icp_batch(w.edges, w.est, p, compute_cov=True)
    ref, ref_h = O.icp_batch(w.pts, w.offsets, w.edges, w.est, p, O.NN_GRID, threads=16)
    _assert_results_equal(res, ref, "config4")
    n = np.diff(w.offsets)
    np.testing.assert_array_equal(hess[:, 0, 0], 2.0 * np.minimum(n[w.edges[:, 1]], n[w.edges[:, 0]]))
    np.testing.assert_allclose(hess, ref_h, rtol=1e-11, atol=1e-7)
    F = w.factors_with_icp(res, p)
    X0 = w.est.astype(np.float64)
    Xg, _ = ctx.optimize_graph(X0, F)
    Xo, _ = O.optimize_graph(X0, F)
    assert np.abs(pose_diff(Xg, Xo)).max() < 1e-6
