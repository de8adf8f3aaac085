"""The angular-index window of the ICP kernel (dpg-slam_amd/csrc/dpg_icp_ang.hip) is exact only if
every target within the search radius falls inside the window.  This restates the device
arithmetic in float32 (pseudo_angle, window half-width) and checks the bound on random queries,
radii and neighbours -- including points right at the radius, near the axes where the octant
polynomial's slope peaks, and a reciprocal carrying a full ulp of error.
"""
import numpy as np

F = np.float32
TWO_PI = F(6.28318530717958647692)
SLOPE, MARGIN = F(1.07), F(2e-5)


def pseudo_angle(x, y, rng):
    x, y = x.astype(F), y.astype(F)
    ax, ay = np.abs(x), np.abs(y)
    mx, mn = np.maximum(ax, ay), np.minimum(ax, ay)
    with np.errstate(divide="ignore", invalid="ignore"):
        r = (F(1) / mx).astype(F)
        r = (r * (F(1) + F(2 ** -23) * rng.choice([F(-1), F(1)], r.shape))).astype(F)   # v_rcp_f32: 1 ulp
        t = (mn * r).astype(F)
    f = (t * (F(1.0584) - F(0.273) * t)).astype(F)
    phi = np.where(ay > ax, F(1.5707963) - f, f).astype(F)
    phi = np.where(x < 0, F(3.14159265) - phi, phi).astype(F)
    phi = np.where(y < 0, TWO_PI - phi, phi).astype(F)
    return np.where(mx > 0, phi, F(0))


def half_width(qx, qy, rad):
    with np.errstate(divide="ignore"):
        sn = (rad * (F(1) / np.sqrt((qx * qx + qy * qy).astype(F))).astype(F) * F(1.0001) + F(1e-6)).astype(F)
    ok = sn < F(0.7)
    s2 = np.where(ok, sn, F(0))
    # the kernel's chord bound of 1/sqrt(1 - sn^2) (dpg_icp_ang.hip window())
    half = (SLOPE * s2 * (s2 * s2 * F(0.8172) + F(1)).astype(F) * F(1.0001) + MARGIN).astype(F)
    return ok, half


def test_window_contains_every_point_within_radius():
    rng = np.random.default_rng(3)
    n = 600_000
    r = np.exp(rng.uniform(np.log(0.05), np.log(30.0), n))
    th = rng.uniform(-np.pi, np.pi, n)
    th[::5] = rng.choice([0.0, np.pi / 2, np.pi, -np.pi / 2, np.pi / 4], n // 5 + (n % 5 > 0))[: len(th[::5])] \
        + rng.normal(0, 1e-3, len(th[::5]))                                   # near the axes / diagonals
    qx, qy = (r * np.cos(th)).astype(F), (r * np.sin(th)).astype(F)
    rho = np.exp(rng.uniform(np.log(1e-5), np.log(0.7), n)).astype(F)
    d = rho * np.sqrt(rng.uniform(0, 1, n))
    d[::3] = rho[::3] * (1 - 1e-7)                                            # on the radius
    a = rng.uniform(-np.pi, np.pi, n)
    px, py = (qx + d * np.cos(a)).astype(F), (qy + d * np.sin(a)).astype(F)
    inside = (px.astype(np.float64) - qx) ** 2 + (py.astype(np.float64) - qy) ** 2 <= rho.astype(np.float64) ** 2
    ok, half = half_width(qx, qy, rho)
    diff = np.abs(pseudo_angle(px, py, rng).astype(np.float64) - pseudo_angle(qx, qy, rng))
    diff = np.minimum(diff, 2 * np.pi - diff)
    sel = inside & ok
    assert sel.sum() > n // 2
    worst = (diff[sel] / half[sel]).max()
    assert not np.any(diff[sel] > half[sel]), f"{np.sum(diff[sel] > half[sel])} points outside the window"
    assert worst < 0.995, worst


def test_pseudo_angle_is_monotone_up_to_float_error():
    rng = np.random.default_rng(4)
    t = np.linspace(0.0, 2 * np.pi, 400_001)[:-1]
    p = pseudo_angle(np.cos(t), np.sin(t), rng).astype(np.float64)
    back = np.diff(p)
    back = back[back > -3.0]                     # drop the wrap at 2 pi
    assert back.min() > -2e-5                    # never steps back by more than the margin
    assert abs(p[-1] - 2 * np.pi) < 1e-3 and p[0] == 0.0
