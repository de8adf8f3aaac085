"""The 6x6 ICP covariance sandwich the reference computes and then discards
(src/icp_cov/cov_func_point_to_point.h:553-566, commented out; ICP_COV is the constant of
:572-575) -- optional, SURVEY §8f rank 4.  Pinned to the reference's OWN generated expressions:
tests/golden/cov6_expr.npz holds every d2J_dX2 and d2J_dZdX entry of the reference evaluated at 400
random points (b = c = z = 0), and the sandwich over three seeded cloud pairs built from them
(tests/golden/make_golden.py).  CPU: the closed forms the kernel and the oracle use (derived
independently, tools/cov6_derive.py) equal the reference's entries; the oracle's sandwich equals the
golden one.  GPU: icp_cov_sandwich (sums on the device, fp64) against the oracle and the golden.

Tolerance: entries agree to 1e-8 of the matrix's largest entry.  The three sides sum the same
terms in different orders and forms (the reference recomputes cos/sin inside each of its generated
expressions; the kernel reduces per-pair closed forms in a 512-lane tree; the oracle sums full 6x6
blocks), and d2J_dX2's yaw and pitch/roll entries are sums of +- terms of magnitude ~1e3 that cancel
to ~1e2, so the inverse carries ~1e-13 absolute (~1e-7 relative on the smallest entries)."""
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "cov6_expr.npz"))


def _closed_forms(a, x, y, p, q):
    ca, sa = np.cos(a), np.sin(a)
    px, py, qx, qy = p[:, 0], p[:, 1], q[:, 0], q[:, 1]
    ux, uy = ca * px - sa * py, sa * px + ca * py
    dx, dy = x - qx, y - qy
    w, v = dx * ca + dy * sa, dx * sa - dy * ca
    n = len(a)
    H, B = np.zeros((n, 6, 6)), np.zeros((n, 6, 6))
    H[:, 0, 0] = H[:, 1, 1] = H[:, 2, 2] = 2.0
    H[:, 0, 3] = H[:, 3, 0] = -2 * uy
    H[:, 1, 3] = H[:, 3, 1] = 2 * ux
    H[:, 2, 4] = H[:, 4, 2] = -2 * px
    H[:, 2, 5] = H[:, 5, 2] = 2 * py
    H[:, 3, 3] = -2 * (ux * dx + uy * dy)
    H[:, 4, 4] = -2 * px * w
    H[:, 4, 5] = H[:, 5, 4] = 2 * py * w
    H[:, 5, 5] = 2 * py * v
    B[:, 0] = np.stack([2 * ca, -2 * sa, 0 * ca, -2 + 0 * ca, 0 * ca, 0 * ca], 1)
    B[:, 1] = np.stack([2 * sa, 2 * ca, 0 * ca, 0 * ca, -2 + 0 * ca, 0 * ca], 1)
    B[:, 2, 2], B[:, 2, 5] = 2.0, -2.0
    B[:, 3] = np.stack([-2 * v, -2 * w, 0 * v, 2 * uy, -2 * ux, 0 * v], 1)
    B[:, 4, 2], B[:, 4, 5] = 2 * w, 2 * px
    B[:, 5, 2], B[:, 5, 5] = 2 * v, -2 * py
    return H, B


def test_closed_forms_equal_reference_expressions():
    H, B = _closed_forms(G["pt_a"], G["pt_x"], G["pt_y"], G["pt_p"], G["pt_q"])
    scale = 1.0 + np.abs(G["pt_H"]).max()
    assert np.abs(H - G["pt_H"]).max() <= 1e-12 * scale
    assert np.abs(B - G["pt_B"]).max() <= 1e-12 * (1.0 + np.abs(G["pt_B"]).max())


@pytest.mark.parametrize("case", [0, 1, 2])
def test_oracle_sandwich_equals_golden(case):
    from oracle import oracle as O
    cov6, cov3 = O.icp_cov_sandwich(G[f"s{case}_p"], G[f"s{case}_q"], G[f"s{case}_T"])
    ref6 = G[f"s{case}_cov6"]
    assert np.abs(cov6 - ref6).max() <= 1e-8 * np.abs(ref6).max()
    np.testing.assert_array_equal(cov3, cov6[np.ix_([0, 1, 3], [0, 1, 3])])


@pytest.mark.gpu
@pytest.mark.parametrize("case", [0, 1, 2])
def test_gpu_sandwich_matches_oracle_and_golden(ctx, case):
    from dpgslam import api
    from oracle import oracle as O
    p, q, T = G[f"s{case}_p"], G[f"s{case}_q"], G[f"s{case}_T"]
    cov6, cov3 = api.icp_cov_sandwich(p, q, T, ctx=ctx)
    o6, o3 = O.icp_cov_sandwich(p, q, T)
    ref6 = G[f"s{case}_cov6"]
    np.testing.assert_allclose(cov6, o6, rtol=1e-9, atol=1e-12 * np.abs(o6).max())
    assert np.abs(cov6 - ref6).max() <= 1e-8 * np.abs(ref6).max()
    np.testing.assert_array_equal(cov3, cov6[np.ix_([0, 1, 3], [0, 1, 3])])


@pytest.mark.gpu
def test_gpu_sandwich_config1(ctx, workload):
    """On the config-1 alignment: the full clouds and the final ICP transform."""
    from dpgslam import api
    from oracle import oracle as O
    w = workload("config1")
    ok, z, cov, res, hess = ctx.run_icp(w.node(0), w.node(1), with_hessian=True)
    T = np.eye(4, dtype=np.float32)
    T[0, 0], T[0, 1], T[0, 3], T[1, 0], T[1, 1], T[1, 3] = res.T
    cov6, cov3 = api.icp_cov_sandwich(w.cloud(1), w.cloud(0), T, ctx=ctx)
    o6, _ = O.icp_cov_sandwich(w.cloud(1), w.cloud(0), T)
    assert np.abs(cov6 - o6).max() <= 1e-8 * np.abs(o6).max()
    # its Hessian's [x, y, yaw] block is the diagnostic block calculate_ICP_COV already returns
    assert np.all(np.isfinite(cov6)) and np.all(np.diag(cov3) > 0)


@pytest.mark.gpu
def test_gpu_sandwich_rejects_non_planar_T(ctx):
    """The closed forms hold at z = pitch = roll = 0; a T with a third row / column that is not
    planar is refused (DPG_ERR_ARG) instead of being evaluated at the wrong operating point."""
    from dpgslam import _abi, api
    p, q, T = G["s0_p"], G["s0_q"], np.asarray(G["s0_T"], np.float32).reshape(4, 4)
    for (r, c, v) in [(2, 3, 0.1), (2, 0, 0.01), (0, 2, 0.01), (2, 2, 0.99)]:
        Tb = T.copy()
        Tb[r, c] = v
        with pytest.raises(_abi.DpgError):
            api.icp_cov_sandwich(p, q, Tb, ctx=ctx)
