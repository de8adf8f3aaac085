"""Golden fixtures (tests/golden/, made by make_golden.py): the oracle reproduces its committed
config-1 vectors bit for bit, and its covariance block matches the reference's own generated
expressions (cov_func_point_to_point.h:133-165) evaluated at the committed inputs."""
import os

import numpy as np

from dpgslam import _abi

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_config1_golden_bit_exact():
    from dpgslam import api
    from oracle import oracle as O
    g = np.load(os.path.join(GOLD, "config1_golden.npz"))
    for v, key in ((0, "cloud0"), (1, "cloud1")):
        c = O.scan_to_cloud(g["ranges"][v], float(g["angle_min"]), float(g["angle_max"]), float(g["range_max"]))
        assert c.tobytes() == g[key].tobytes()
    for ratio in (5, 1):
        p = _abi.default_icp_params()
        p.downsample_icp_points_ratio = ratio
        sd, td = api.downsample(g["cloud1"], ratio), api.downsample(g["cloud0"], ratio)
        guess = O.icp_guess(g["est"][1], g["est"][0])
        assert guess.tobytes() == g[f"r{ratio}_guess"].tobytes()
        res, tr = O.icp_align(sd, td, guess, p, O.NN_BRUTE, trace_iters=100)
        assert bytes(res) == g[f"r{ratio}_result"].tobytes()
        np.testing.assert_array_equal(tr[:res.iterations], g[f"r{ratio}_trace"])
        cov, hess = O.icp_cov(g["cloud1"], g["cloud0"], np.array(res.T, np.float32))
        assert cov.tobytes() == g[f"r{ratio}_cov"].tobytes()
        np.testing.assert_allclose(hess, g[f"r{ratio}_hess"], rtol=1e-14)


def test_cov_block_matches_reference_expressions():
    """Closed form of the [x,y,yaw] block == the reference's generated d2J expressions."""
    d = np.load(os.path.join(GOLD, "cov_expr.npz"))
    a, x, y = d["a"], d["x"], d["y"]
    ux = np.cos(a) * d["pix"] - np.sin(a) * d["piy"]
    uy = np.sin(a) * d["pix"] + np.cos(a) * d["piy"]
    rx, ry = (x - d["qix"]) + ux, (y - d["qiy"]) + uy
    np.testing.assert_allclose(-2.0 * uy, d["d2J_dxda"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(2.0 * ux, d["d2J_dyda"], rtol=1e-12, atol=1e-12)
    da2 = 2.0 * (ux * ux + uy * uy) - 2.0 * (ux * rx + uy * ry)
    np.testing.assert_allclose(da2, d["d2J_da2"], rtol=1e-11, atol=1e-9)
    # and the oracle's per-point accumulation uses exactly that closed form
    from oracle import oracle as O
    for k in range(0, 400, 37):
        T6 = np.array([np.cos(a[k]), -np.sin(a[k]), x[k], np.sin(a[k]), np.cos(a[k]), y[k]], np.float32)
        p = np.array([[d["pix"][k], d["piy"][k]]], np.float32)
        q = np.array([[d["qix"][k], d["qiy"][k]]], np.float32)
        _, h = O.icp_cov(p, q, T6)
        _, hl = O.icp_cov(p, q, T6, literal=True)
        np.testing.assert_allclose(h, hl, rtol=1e-11, atol=1e-9)
