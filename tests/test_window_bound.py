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


def _f32_fma(a, b, c):
    """fmaf in float32: the float64 product of two float32 values is exact, so one rounding of the
    float64 sum is the fused result (for these magnitudes)."""
    return (a.astype(np.float64) * b.astype(np.float64) + np.float64(c)).astype(F)


def test_variant5_window_contains_every_point_within_radius():
    """The default kernel form (variant 5): the query's pseudo-angle in bucket units (the scale folded
    into the octant polynomial's constants) and the half-width's margins folded into three
    constants (window_pa).  Every cloud point within the radius must land, through the BUILD side's
    bucket map floor(pseudo_angle(p) * scale), inside [floor(ps - hs), floor(ps + hs)] modulo the
    bucket count."""
    rng = np.random.default_rng(5)
    kB = 1024
    S = F(F(kB) / TWO_PI)
    A, B = F(F(1.0584) * S), F(F(0.273) * S)
    Q1, Q2, Q4 = F(F(1.5707963) * S), F(F(3.14159265) * S), F(TWO_PI * S)
    QUAD, SL, MG = F(F(0.8172) * F(1.001)), F(F(1.07) * F(1.0003) * S), F((MARGIN + F(2e-6)) * S)
    n = 600_000
    r = np.exp(rng.uniform(np.log(0.05), np.log(30.0), n))
    th = rng.uniform(-np.pi, np.pi, n)
    th[::5] = rng.choice([0.0, np.pi / 2, np.pi, -np.pi / 2, np.pi / 4], n // 5 + (n % 5 > 0))[: len(th[::5])] \
        + rng.normal(0, 1e-3, len(th[::5]))
    qx, qy = (r * np.cos(th)).astype(F), (r * np.sin(th)).astype(F)
    rho = np.exp(rng.uniform(np.log(1e-5), np.log(0.7), n)).astype(F)
    d = rho * np.sqrt(rng.uniform(0, 1, n))
    d[::3] = rho[::3] * (1 - 1e-7)
    a = rng.uniform(-np.pi, np.pi, n)
    px, py = (qx + d * np.cos(a)).astype(F), (qy + d * np.sin(a)).astype(F)
    inside = (px.astype(np.float64) - qx) ** 2 + (py.astype(np.float64) - qy) ** 2 <= rho.astype(np.float64) ** 2
    # query side (pseudo_angle_b): v_rcp_f32 with one ulp of error either way
    ax, ay = np.abs(qx), np.abs(qy)
    mx, mn = np.maximum(ax, ay), np.minimum(ax, ay)
    rc = (F(1) / mx).astype(F)
    rc = (rc * (F(1) + F(2 ** -23) * rng.choice([F(-1), F(1)], n))).astype(F)
    t = (mn * rc).astype(F)
    f = (t * (A - (B * t).astype(F)).astype(F)).astype(F)
    ps = np.where(ay > ax, (Q1 - f).astype(F), f).astype(F)
    ps = np.where(qx < 0, (Q2 - ps).astype(F), ps).astype(F)
    ps = np.where(qy < 0, (Q4 - ps).astype(F), ps).astype(F)
    # window_pa<5>: s0 = rad * v_rsq_f32(|q|^2) (one ulp), hs = fma(s0 * fma(s0^2, QUAD, 1), SL, MG)
    q2 = ((qx * qx).astype(F) + (qy * qy).astype(F)).astype(F)
    rs = (F(1) / np.sqrt(q2)).astype(F)
    rs = (rs * (F(1) + F(2 ** -23) * rng.choice([F(-1), F(1)], n))).astype(F)
    s0 = (rho * rs).astype(F)
    ok = s0 < F(0.6999)
    hs = _f32_fma((s0 * _f32_fma((s0 * s0).astype(F), QUAD, 1.0)).astype(F), SL, MG)
    blo = np.floor((ps - hs).astype(F)).astype(np.int64)
    bhi = np.floor((ps + hs).astype(F)).astype(np.int64)
    # build side (angle_index_kernel): bucket_of(pseudo_angle(p)) in radians, then the scale
    bp = np.clip(np.floor((pseudo_angle(px, py, rng) * S).astype(F)).astype(np.int64), 0, kB - 1)
    wrap = (blo < 0) | (bhi >= kB)
    lo, hi = blo % kB, bhi % kB
    within = np.where(wrap, (bp >= lo) | (bp <= hi), (bp >= lo) & (bp <= hi))
    sel = inside & ok
    assert sel.sum() > n // 2
    assert within[sel].all(), f"{np.sum(~within[sel])} points outside the variant-5 window"
    # and the continuous bound itself, in bucket units, with room to spare
    diff = np.abs(pseudo_angle(px, py, rng).astype(np.float64) * np.float64(S) - ps)
    diff = np.minimum(diff, kB - diff)
    worst = (diff[sel] / hs[sel]).max()
    assert worst < 0.995, worst
