"""CPU tests of the oracle (test infrastructure) against the reference's own known answers and
independent checks (no GPU needed)."""
import math

import numpy as np
import pytest

from graphs import gtsam_test_graph, pose_diff


def O():
    from oracle import oracle
    return oracle


def test_gtsam_test_known_answer():
    """dpg_slam_main.cc:224-251: the consistent 2 m square; optimum known analytically."""
    from dpgslam import _abi
    X0, F, X_opt = gtsam_test_graph()
    for crit in (0, 1):
        gp = _abi.default_gn_params()
        gp.use_error_criteria = crit
        X, st = O().optimize_graph(X0, F, gp)
        assert np.abs(pose_diff(X, X_opt)).max() < 1e-9
        assert st.final_error < 1e-12
    # GTSAM GaussNewtonParams (relativeErrorTol 1e-5): converges in a handful of iterations
    assert st.iterations <= 6


def _square_scan(n=720, seed=0):
    """A closed room scan (rectangle + a box) as seen from inside, noiseless."""
    rng = np.random.default_rng(seed)
    a = np.linspace(-np.pi, np.pi, n, endpoint=False)
    d = np.stack([np.cos(a), np.sin(a)], 1)
    W, H = 6.0 + rng.random(), 4.0 + rng.random()
    ox, oy = 0.4, -0.3
    t = np.full(n, np.inf)
    for (px, py, vx, vy) in [(-W / 2, -H / 2, W, 0), (W / 2, -H / 2, 0, H), (W / 2, H / 2, -W, 0), (-W / 2, H / 2, 0, -H),
                             (1.0, 0.5, 0.6, 0), (1.6, 0.5, 0, 0.5), (1.6, 1.0, -0.6, 0), (1.0, 1.0, 0, -0.5)]:
        den = d[:, 0] * vy - d[:, 1] * vx
        with np.errstate(divide="ignore", invalid="ignore"):
            wx, wy = px - ox, py - oy
            tt = (wx * vy - wy * vx) / den
            uu = (wx * d[:, 1] - wy * d[:, 0]) / den
        ok = (np.abs(den) > 1e-12) & (tt > 0) & (uu >= 0) & (uu <= 1)
        t = np.where(ok & (tt < t), tt, t)
    return (d * t[:, None]).astype(np.float32)


@pytest.mark.parametrize("theta,tx,ty", [(0.0, 0.0, 0.0), (0.1, 0.2, -0.1), (-0.2, -0.25, 0.3), (0.15, 0.05, 0.05)])
def test_icp_recovers_known_transform(theta, tx, ty):
    """a scan and its copy under a known rigid motion (theta <= 0.2 rad), no noise:
    from a guess off by (0.002 rad, 1 cm) -- as runIcp's odometry guess is -- ICP returns the
    motion within 1e-5 m / 1e-6 rad.  (From far guesses point-to-point ICP on a regularly sampled
    scan has local minima about one beam step of rotation away; PCL shares them.)"""
    from dpgslam import _abi
    tgt = _square_scan()
    c, s = math.cos(theta), math.sin(theta)
    # source = T^-1 (target) so that T * source = target
    src = ((tgt - np.array([tx, ty], np.float32)) @ np.array([[c, -s], [s, c]], np.float32)).astype(np.float32)
    p = _abi.default_icp_params()
    g0 = theta + 0.002
    guess = np.array([math.cos(g0), -math.sin(g0), tx + 0.01, math.sin(g0), math.cos(g0), ty - 0.01], np.float32)
    res, _ = O().icp_align(src, tgt, guess, p, O().NN_GRID)
    assert res.converged and res.status == 0
    assert abs(res.z[0] - tx) < 1e-5 and abs(res.z[1] - ty) < 1e-5
    assert abs(math.atan2(math.sin(res.z[2] - theta), math.cos(res.z[2] - theta))) < 1e-6


def test_grid_nn_equals_brute_force(workload):
    """The oracle's grid 1-NN gives the exact brute-force result (same float distances, lowest
    index on ties) -- checked on whole ICP runs of config-2 edges and on tie-heavy inputs."""
    from dpgslam import _abi, api
    w = workload("config2")
    p = _abi.default_icp_params()
    for e in range(0, w.E, 50):
        t, s = w.edges[e]
        sd, td = api.downsample(w.cloud(s), 5), api.downsample(w.cloud(t), 5)
        g = api.icp_guess(w.est[s], w.est[t])
        rb, tb = O().icp_align(sd, td, g, p, O().NN_BRUTE, trace_iters=30)
        rg, tg = O().icp_align(sd, td, g, p, O().NN_GRID, trace_iters=30)
        assert bytes(rb) == bytes(rg)
        np.testing.assert_array_equal(tb, tg)
    # exact ties: duplicated target points (ties must go to the lowest index)
    tgt = np.repeat(_square_scan(180), 3, axis=0)
    src = tgt[::3] + np.float32(0.01)
    p.icp_maximum_iterations = 5
    rb, tb = O().icp_align(src, tgt, np.array([1, 0, 0, 0, 1, 0], np.float32), p, O().NN_BRUTE, trace_iters=5)
    rg, tg = O().icp_align(src, tgt, np.array([1, 0, 0, 0, 1, 0], np.float32), p, O().NN_GRID, trace_iters=5)
    np.testing.assert_array_equal(tb, tg)
    assert (tb[0][tb[0] >= 0] % 3 == 0).all()


def test_forward_nn_matches_scipy(workload):
    """First-iteration correspondences: every accepted pair is the scipy cKDTree 1-NN (ties aside)."""
    from scipy.spatial import cKDTree
    from dpgslam import _abi, api
    w = workload("config2")
    p = _abi.default_icp_params()
    t, s = w.edges[7]
    sd, td = api.downsample(w.cloud(s), 5), api.downsample(w.cloud(t), 5)
    g = api.icp_guess(w.est[s], w.est[t])
    _, tr = O().icp_align(sd, td, g, p, O().NN_BRUTE, trace_iters=1)
    src0 = np.stack([(g[0] * sd[:, 0] + g[1] * sd[:, 1]) + g[2], (g[3] * sd[:, 0] + g[4] * sd[:, 1]) + g[5]], 1)
    src0 = src0.astype(np.float32)
    d, j = cKDTree(td.astype(np.float64)).query(src0.astype(np.float64))
    acc = tr[0] >= 0
    assert acc.sum() > 0.5 * len(sd)
    agree = (tr[0][acc] == j[acc]) | np.isclose(d[acc], np.linalg.norm(src0[acc] - td[tr[0][acc]], axis=1))
    assert agree.all()
    # reciprocity: accepted pairs are mutual nearest neighbours
    d2, i2 = cKDTree(src0.astype(np.float64)).query(td[tr[0][acc]].astype(np.float64))
    assert (i2 == np.nonzero(acc)[0]).mean() > 0.999


def test_cov_block_closed_form_equals_literal(workload):
    """The oracle's closed-form [x,y,yaw] block equals a symbol-by-symbol evaluation of the
    reference expressions (cov :133-165) at b = c = z = 0."""
    w = workload("config1")
    T6 = np.array([0.93, -0.36, 0.4, 0.36, 0.93, -0.2], np.float32)
    _, h = O().icp_cov(w.cloud(1), w.cloud(0), T6)
    _, hl = O().icp_cov(w.cloud(1), w.cloud(0), T6, literal=True)
    np.testing.assert_allclose(h, hl, rtol=1e-12, atol=1e-9)


def test_cov_constant_output():
    """ICP_COV = diag(var_x, var_y, var_theta) widened from float (cov :572-575)."""
    pts = np.zeros((3, 2), np.float32)
    cov, _ = O().icp_cov(pts, pts, np.array([1, 0, 0, 0, 1, 0], np.float32), 0.5, 0.5, 0.3)
    assert cov.tobytes() == np.diag([0.5, 0.5, float(np.float32(0.3))]).tobytes()


def _num_jac(fun, X, k, eps=1e-6):
    """d e / d (right perturbation of pose k through the cheap Pose2 retract)."""
    from dpgslam.synth import _compose
    J = np.zeros((3, 3))
    for c in range(3):
        d = np.zeros(3)
        d[c] = eps
        Xp, Xm = X.copy(), X.copy()
        Xp[k] = _compose(X[k], d)
        Xm[k] = _compose(X[k], -d)
        ep, em = fun(Xp), fun(Xm)
        diff = ep - em
        diff[2] = math.atan2(math.sin(diff[2]), math.cos(diff[2]))
        J[:, c] = diff / (2 * eps)
    return J


def test_between_jacobians_finite_differences():
    """BetweenFactor<Pose2>: A_i / A_j are Pose2::between's Jacobians (GTSAM default, no
    SLOW_BUT_CORRECT_BETWEENFACTOR): de/dX = L(d) A with L(d) = blkdiag(R(d_theta), 1), d = z^-1 h."""
    from dpgslam import api
    rng = np.random.default_rng(3)
    for _ in range(20):
        X = rng.normal(0, 2, (2, 3))
        X[:, 2] = rng.uniform(-3, 3, 2)
        f = api.between_factor(0, 1, rng.normal(0, 1, 3), (0.1, 0.1, 0.1))[0]
        e, Ai, Aj = O().linearize(f, X)
        fun = lambda Y: O().linearize(f, Y)[0]
        Ld = np.eye(3)
        c, s = math.cos(e[2]), math.sin(e[2])
        Ld[:2, :2] = [[c, -s], [s, c]]
        np.testing.assert_allclose(_num_jac(fun, X, 0), Ld @ Ai, atol=1e-7)
        np.testing.assert_allclose(_num_jac(fun, X, 1), Ld @ Aj, atol=1e-7)
        np.testing.assert_array_equal(Aj, np.eye(3))


def test_prior_jacobian_at_optimum():
    """PriorFactor<Pose2>: e = -Local(x, prior), H = I (exact at x = prior)."""
    from dpgslam import api
    P = np.array([0.3, -0.2, 0.7])
    f = api.prior_factor(0, tuple(P), (0.2, 0.2, 0.15))[0]
    X = P[None, :].copy()
    e, Ai, _ = O().linearize(f, X)
    assert np.abs(e).max() < 1e-15
    np.testing.assert_allclose(_num_jac(lambda Y: O().linearize(f, Y)[0], X, 0), Ai, atol=1e-7)


def test_oracle_gn_converges_config3(workload):
    """Block-sparse Cholesky GN on config 3 (with oracle ICP results): converges, error drops."""
    w = workload("config3")
    from dpgslam import _abi
    p = _abi.default_icp_params()
    res, _ = O().icp_batch(w.pts, w.offsets, w.edges, w.est, p, O().NN_GRID, threads=8)
    F = w.factors_with_icp(res, p)
    X, st = O().optimize_graph(w.est.astype(np.float64), F)
    assert st.iterations < 30 and st.last_delta_inf < 1e-10
    assert st.final_error < st.initial_error
    # one more GN step from the optimum moves nothing
    d, _ = O().gn_delta(X, F)
    assert np.abs(d).max() < 1e-9
