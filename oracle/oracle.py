"""TEST INFRASTRUCTURE ONLY -- ctypes loader for the CPU oracle (oracle/build/liboracle.so).

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the CHECKER (and the
timed CPU baseline, kind "port"); never by the product path.  See dpg_oracle.h for what is
pinned by the reference's own known answers and what is unpinned (PCL / GTSAM arithmetic).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")

NN_BRUTE = 0
NN_GRID = 1

_L = None


def build():
    subprocess.run(["make", "-C", _HERE], check=True, stdout=subprocess.DEVNULL)


def lib():
    global _L
    if _L is None:
        if not os.path.exists(LIB_PATH):
            build()
        from dpgslam import _abi
        L = C.CDLL(LIB_PATH)
        F32P, F64P, I32P, I64P, P = _abi.F32P, _abi.F64P, _abi.I32P, _abi.I64P, C.c_void_p
        sig = {
            "oracle_scan_to_cloud": (C.c_int64, [F32P, C.c_int64, C.c_float, C.c_float, C.c_float, C.c_float,
                                                 C.c_float, C.c_float, F32P]),
            "oracle_downsample": (C.c_int64, [F32P, C.c_int64, C.c_int32, F32P]),
            "oracle_inverse_transform_point": (None, [F32P, F32P, F32P]),
            "oracle_transform_point": (None, [F32P, F32P, F32P]),
            "oracle_icp_guess": (None, [F32P, F32P, F32P]),
            "oracle_icp_align": (C.c_int, [F32P, C.c_int64, F32P, C.c_int64, F32P, C.POINTER(_abi.IcpParams),
                                           C.c_int, C.POINTER(_abi.IcpResult), I32P, C.c_int32]),
            "oracle_icp_cov": (None, [F32P, C.c_int64, F32P, C.c_int64, F32P, C.c_float, C.c_float, C.c_float,
                                      F64P, F64P]),
            "oracle_cov_block_literal": (None, [F32P, C.c_int64, F32P, C.c_int64, F32P, F64P]),
            "oracle_run_icp": (C.c_int, [F32P, C.c_int64, F32P, C.c_int64, F32P, F32P, C.POINTER(_abi.IcpParams),
                                         C.c_int, C.POINTER(_abi.IcpResult), F64P, F64P]),
            "oracle_icp_batch": (C.c_int, [F32P, I64P, C.c_int64, I32P, C.c_int64, F32P, C.POINTER(_abi.IcpParams),
                                           C.c_int, C.c_int, P, F64P]),
            "oracle_linearize": (None, [P, F64P, F64P, F64P, F64P]),
            "oracle_graph_error": (C.c_double, [F64P, P, C.c_int64]),
            "oracle_optimize_graph": (C.c_int, [F64P, C.c_int64, P, C.c_int64, C.POINTER(_abi.GnParams),
                                                C.POINTER(_abi.GnStats)]),
            "oracle_gn_delta": (C.c_int, [F64P, C.c_int64, P, C.c_int64, F64P, F64P]),
            "oracle_dpg_create": (P, [C.c_int64, I64P, F32P, F32P, C.POINTER(_abi.ChangeParams)]),
            "oracle_dpg_destroy": (None, [P]),
            "oracle_dpg_append": (C.c_int, [P, C.c_int64, I64P, F32P, F32P]),
            "oracle_execute_dpg": (C.c_int, [P, C.c_int64, C.c_int64, F32P, C.POINTER(_abi.ChangeStats)]),
            "oracle_execute_dpg_chain": (C.c_int, [P, C.c_int64, C.c_int64, F32P, F32P, C.POINTER(_abi.ChangeStats)]),
            "oracle_dpg_fetch": (None, [P, _abi.U8P, _abi.U8P, _abi.U8P]),
            "oracle_dpg_load": (None, [P, _abi.U8P, _abi.U8P, _abi.U8P]),
            "oracle_active_dynamic_points": (C.c_int64, [P, C.c_int64, F32P, F32P, C.c_int64, I64P]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _L = L
    return _L


def _p(a, t):
    return None if a is None else a.ctypes.data_as(C.POINTER(t))


def _f32(a):
    return np.ascontiguousarray(np.asarray(a, np.float32))


def scan_to_cloud(ranges, amin, amax, rmax, laser=(0.2, 0.0, 0.0)):
    r = _f32(ranges)
    out = np.empty((max(r.size, 1), 2), np.float32)
    n = lib().oracle_scan_to_cloud(_p(r, C.c_float), r.size, amin, amax, rmax, *laser, _p(out, C.c_float))
    return out[:n].copy()


def downsample(cloud, ratio):
    c = _f32(cloud).reshape(-1, 2)
    out = np.empty((max(len(c), 1), 2), np.float32)
    n = lib().oracle_downsample(_p(c, C.c_float), len(c), ratio, _p(out, C.c_float))
    return out[:n].copy()


def inverse_transform_point(a, b):
    a, b, o = _f32(a), _f32(b), np.empty(3, np.float32)
    lib().oracle_inverse_transform_point(_p(a, C.c_float), _p(b, C.c_float), _p(o, C.c_float))
    return o


def transform_point(p, f):
    p, f, o = _f32(p), _f32(f), np.empty(3, np.float32)
    lib().oracle_transform_point(_p(p, C.c_float), _p(f, C.c_float), _p(o, C.c_float))
    return o


def icp_guess(ps, pt):
    a, b, o = _f32(ps), _f32(pt), np.empty(6, np.float32)
    lib().oracle_icp_guess(_p(a, C.c_float), _p(b, C.c_float), _p(o, C.c_float))
    return o


def icp_align(src_ds, tgt_ds, guess, params=None, nn=NN_BRUTE, trace_iters=0):
    """PCL ICP align on downsampled clouds. Returns (IcpResult, trace [iters, n_src] or None)."""
    from dpgslam import _abi
    p = params or _abi.default_icp_params()
    s, t, g = _f32(src_ds).reshape(-1, 2), _f32(tgt_ds).reshape(-1, 2), _f32(guess)
    res = _abi.IcpResult()
    tr = np.full((trace_iters, len(s)), -1, np.int32) if trace_iters else None
    lib().oracle_icp_align(_p(s, C.c_float), len(s), _p(t, C.c_float), len(t), _p(g, C.c_float), C.byref(p), nn,
                           C.byref(res), _p(tr, C.c_int32), trace_iters)
    return res, tr


def icp_cov(data, model, T6, vx=0.5, vy=0.5, vth=0.3, literal=False):
    d, m, T = _f32(data).reshape(-1, 2), _f32(model).reshape(-1, 2), _f32(T6)
    cov, hess = np.zeros(9), np.zeros(9)
    if literal:
        lib().oracle_cov_block_literal(_p(d, C.c_float), len(d), _p(m, C.c_float), len(m), _p(T, C.c_float),
                                       _p(hess, C.c_double))
        return None, hess.reshape(3, 3)
    lib().oracle_icp_cov(_p(d, C.c_float), len(d), _p(m, C.c_float), len(m), _p(T, C.c_float), vx, vy, vth,
                         _p(cov, C.c_double), _p(hess, C.c_double))
    return cov.reshape(3, 3), hess.reshape(3, 3)


def icp_cov_sandwich(data, model, T4):
    """The commented-out 6x6 sandwich (cov :553-566): (cov6 [6, 6], cov3 [3, 3]); T4 row-major 4x4."""
    d, m = _f32(data).reshape(-1, 2), _f32(model).reshape(-1, 2)
    T = np.asarray(T4, np.float32).reshape(4, 4)
    T6 = np.ascontiguousarray([T[0, 0], T[0, 1], T[0, 3], T[1, 0], T[1, 1], T[1, 3]], np.float32)
    cov6, cov3 = np.zeros(36), np.zeros(9)
    rc = lib().oracle_icp_cov_sandwich(_p(d, C.c_float), len(d), _p(m, C.c_float), len(m), _p(T6, C.c_float),
                                       _p(cov6, C.c_double), _p(cov3, C.c_double))
    if rc:
        raise ValueError(f"oracle_icp_cov_sandwich failed ({rc})")
    return cov6.reshape(6, 6), cov3.reshape(3, 3)


def run_icp(src_full, tgt_full, pose_src, pose_tgt, params=None, nn=NN_GRID):
    from dpgslam import _abi
    p = params or _abi.default_icp_params()
    s, t = _f32(src_full).reshape(-1, 2), _f32(tgt_full).reshape(-1, 2)
    a, b = _f32(pose_src), _f32(pose_tgt)
    res = _abi.IcpResult()
    cov, hess = np.zeros(9), np.zeros(9)
    lib().oracle_run_icp(_p(s, C.c_float), len(s), _p(t, C.c_float), len(t), _p(a, C.c_float), _p(b, C.c_float),
                         C.byref(p), nn, C.byref(res), _p(cov, C.c_double), _p(hess, C.c_double))
    return res, cov.reshape(3, 3), hess.reshape(3, 3)


def icp_batch(pts, offsets, edges, poses, params=None, nn=NN_GRID, threads=1):
    from dpgslam import _abi
    p = params or _abi.default_icp_params()
    pts, offs = _f32(pts).reshape(-1, 2), np.ascontiguousarray(offsets, np.int64)
    e = np.ascontiguousarray(edges, np.int32).reshape(-1, 2)
    ps = _f32(poses).reshape(-1, 3)
    res = np.zeros(len(e), _abi.RESULT_DTYPE)
    hess = np.zeros((len(e), 9))
    lib().oracle_icp_batch(_p(pts, C.c_float), _p(offs, C.c_int64), len(offs) - 1, _p(e, C.c_int32), len(e),
                           _p(ps, C.c_float), C.byref(p), nn, threads, C.c_void_p(res.ctypes.data),
                           _p(hess, C.c_double))
    return res, hess.reshape(-1, 3, 3)


def linearize(factor, poses):
    from dpgslam import _abi
    f = np.ascontiguousarray(np.asarray(factor, _abi.FACTOR_DTYPE).reshape(1))
    X = np.ascontiguousarray(poses, np.float64)
    e, Ai, Aj = np.zeros(3), np.zeros(9), np.zeros(9)
    lib().oracle_linearize(C.c_void_p(f.ctypes.data), _p(X, C.c_double), _p(e, C.c_double), _p(Ai, C.c_double),
                           _p(Aj, C.c_double))
    return e, Ai.reshape(3, 3), Aj.reshape(3, 3)


def graph_error(poses, factors):
    from dpgslam import _abi
    X = np.ascontiguousarray(poses, np.float64)
    F = np.ascontiguousarray(factors, _abi.FACTOR_DTYPE)
    return lib().oracle_graph_error(_p(X, C.c_double), C.c_void_p(F.ctypes.data), len(F))


def optimize_graph(poses, factors, params=None):
    from dpgslam import _abi
    X = np.ascontiguousarray(poses, np.float64).reshape(-1, 3).copy()
    F = np.ascontiguousarray(factors, _abi.FACTOR_DTYPE)
    gp = params or _abi.default_gn_params()
    st = _abi.GnStats()
    rc = lib().oracle_optimize_graph(_p(X, C.c_double), len(X), C.c_void_p(F.ctypes.data), len(F), C.byref(gp),
                                     C.byref(st))
    if rc:
        raise RuntimeError(f"oracle_optimize_graph failed ({rc})")
    return X, st


def gn_delta(poses, factors):
    from dpgslam import _abi
    X = np.ascontiguousarray(poses, np.float64).reshape(-1, 3)
    F = np.ascontiguousarray(factors, _abi.FACTOR_DTYPE)
    d, err = np.zeros(X.size), C.c_double(0)
    rc = lib().oracle_gn_delta(_p(X, C.c_double), len(X), C.c_void_p(F.ctypes.data), len(F), _p(d, C.c_double),
                               C.byref(err))
    if rc:
        raise RuntimeError(f"oracle_gn_delta failed ({rc})")
    return d.reshape(-1, 3), err.value


def loop_closure_candidates(est, passes, within=5.0, across=2.0):
    """reoptimize's candidate pairs (dpg_slam.cc:91-98): for i ascending, j = 0 .. i-2 ascending,
    (j, i) when the float32 (p_j - p_i).norm() (Eigen Vector2f: sqrt(dx*dx + dy*dy), correctly
    rounded) is <= within (same pass, parameters.h:212) or <= across (parameters.h:224)."""
    e = _f32(est).reshape(-1, 3)
    ps = np.asarray(passes, np.int64)
    out = []
    for i in range(2, len(e)):
        d = e[:i - 1, :2] - e[i, :2]
        dist = np.sqrt(d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1])
        thr = np.where(ps[:i - 1] == ps[i], np.float32(within), np.float32(across))
        js = np.nonzero(dist <= thr)[0]
        out.extend((int(j), i) for j in js)
    return np.array(out, np.int32).reshape(-1, 2)


def odometry_factor(odom_prev, odom_cur, i_prev, i_cur, motion=(0.4, 0.4, 0.4, 0.4)):
    """The odometry Between of reoptimize (dpg_slam.cc:55-75): displacement by
    inverseTransformPoint, sigmas from the motion model in float, Diagonal::Sigmas -> 1/sigma^2."""
    from dpgslam import _abi
    d = inverse_transform_point(_f32(odom_cur), _f32(odom_prev))
    f32 = np.float32
    norm = np.sqrt(f32(d[0]) * f32(d[0]) + f32(d[1]) * f32(d[1]))
    m = [f32(x) for x in motion]
    st = f32(m[0] * norm) + f32(m[1] * np.abs(f32(d[2])))
    sr = f32(m[2] * norm) + f32(m[3] * np.abs(f32(d[2])))
    f = np.zeros(1, _abi.FACTOR_DTYPE)
    f["kind"], f["i"], f["j"] = _abi.DPG_FACTOR_BETWEEN, i_prev, i_cur
    f["z"] = np.asarray(d, np.float32).astype(np.float64)
    st, sr = float(st), float(sr)
    f["info"] = [1.0 / (st * st), 1.0 / (st * st), 1.0 / (sr * sr)]
    return f


def reoptimize(pts, offsets, passes, est, odom, icp_params=None, gn_params=None, within=5.0, across=2.0,
               prior_sigmas=(0.2, 0.2, 0.15), threads=1):
    """DpgSLAM::reoptimize (dpg_slam.cc:35-120), restated: per node a prior on the first node of a
    pass or the odometry Between; the successive alignment (always a factor) and every loop-closure
    candidate (a factor when converged); batch GN from the estimated poses.  The oracle ICP aligns
    every edge (grid NN); returns (poses, edges, results)."""
    from dpgslam import _abi
    e = _f32(est).reshape(-1, 3)
    V = len(e)
    p = icp_params or _abi.default_icp_params()
    lc = loop_closure_candidates(e, passes, within, across)
    succ = np.stack([np.arange(V - 1), np.arange(1, V)], 1).astype(np.int32)
    edges = np.concatenate([succ, lc], 0).astype(np.int32)
    res, _ = icp_batch(pts, offsets, edges, e, p, NN_GRID, threads)
    F = []
    cur = None
    for i in range(V):
        if i == 0 or passes[i] != cur:
            f = np.zeros(1, _abi.FACTOR_DTYPE)
            f["kind"], f["i"] = _abi.DPG_FACTOR_PRIOR, i
            s = np.asarray(prior_sigmas, np.float32).astype(np.float64)
            f["info"] = 1.0 / (s * s)
            F.append(f)
            cur = passes[i]
        else:
            F.append(odometry_factor(odom[i - 1], odom[i], i - 1, i))
    info = np.array([1.0 / float(np.float32(p.laser_x_variance)), 1.0 / float(np.float32(p.laser_y_variance)),
                     1.0 / float(np.float32(p.laser_theta_variance))])
    for k, (a, b) in enumerate(edges):
        keep = k < len(succ) or (res["converged"][k] != 0 and res["status"][k] == _abi.DPG_ICP_OK)
        if keep:
            f = np.zeros(1, _abi.FACTOR_DTYPE)
            f["kind"], f["i"], f["j"] = _abi.DPG_FACTOR_BETWEEN, a, b
            f["z"] = res["z"][k].astype(np.float64)
            f["info"] = info
            F.append(f)
    X, st = optimize_graph(e.astype(np.float64), np.concatenate(F), gn_params)
    return X, edges, res, st


def get_map(pts, offsets, est, fraction=10):
    """DpgSLAM::GetMap (dpg_slam.cc:555-575): every node's base_link point in the map frame by
    math_utils::transformPoint (Rotation2Df(angle) * p + pos, float; cos/sin as cosf/sinf), one in
    `fraction` by the running point index over all nodes (display_points_fraction_)."""
    p = _f32(pts).reshape(-1, 2)
    e = _f32(est).reshape(-1, 3)
    offs = np.asarray(offsets, np.int64)
    keep = np.arange(0, offs[-1], fraction)
    node = np.searchsorted(offs, keep, side="right") - 1
    c = np.array([_cos_sin(e[v, 2]) for v in range(len(e))], np.float32)
    x, y = p[keep, 0], p[keep, 1]
    cc, ss = c[node, 0], c[node, 1]
    rx = cc * x + (-ss) * y
    ry = ss * x + cc * y
    return np.stack([e[node, 0] + rx, e[node, 1] + ry], 1).astype(np.float32)


def _cos_sin(th):
    """cosf/sinf of a float angle via the oracle's C transformPoint of unit vectors."""
    a = transform_point(np.array([1.0, 0.0, 0.0], np.float32), np.array([0.0, 0.0, th], np.float32))
    return a[0], a[1]


class OracleDpgStore:
    """CPU restatement of the DPG node store + executeDPG (dpg_change_oracle.cpp); same interface as
    dpgslam.api.DpgStore."""

    def __init__(self, ranges, geom, offsets=None, params=None):
        from dpgslam import _abi
        r = _f32(ranges)
        if offsets is None:
            V, nb = r.shape
            offsets = np.arange(V + 1, dtype=np.int64) * nb
        off = np.ascontiguousarray(offsets, np.int64)
        self.V, self.B = len(off) - 1, int(off[-1])
        g = _f32(geom).reshape(self.V, 3)
        self.params = params or _abi.default_change_params_host()
        self.handle = lib().oracle_dpg_create(self.V, _p(off, C.c_int64), _p(r.reshape(-1), C.c_float),
                                              _p(g, C.c_float), C.byref(self.params))

    def __del__(self):
        if getattr(self, "handle", None):
            lib().oracle_dpg_destroy(self.handle)
            self.handle = None

    def execute_dpg(self, n_nodes, current_pass_len, est, chain_poses=None):
        """chain_poses [chain_n][3]: the current_pass_nodes_ copies' poses (dpg_slam.cc:598), or None."""
        from dpgslam import _abi
        e = _f32(est).reshape(-1, 3)
        st = _abi.ChangeStats()
        if chain_poses is None:
            rc = lib().oracle_execute_dpg(self.handle, n_nodes, current_pass_len, _p(e, C.c_float), C.byref(st))
        else:
            c = _f32(chain_poses).reshape(-1, 3)
            rc = lib().oracle_execute_dpg_chain(self.handle, n_nodes, current_pass_len, _p(e, C.c_float),
                                                _p(c, C.c_float), C.byref(st))
        assert rc == 0, rc
        return st

    def append(self, ranges, geom, offsets=None):
        r = _f32(ranges)
        if offsets is None:
            n, nb = r.shape
            offsets = np.arange(n + 1, dtype=np.int64) * nb
        off = np.ascontiguousarray(offsets, np.int64)
        g = _f32(geom).reshape(-1, 3)
        lib().oracle_dpg_append(self.handle, len(off) - 1, _p(off, C.c_int64), _p(r.reshape(-1), C.c_float),
                                _p(g, C.c_float))
        self.V += len(off) - 1
        self.B += int(off[-1] - off[0])

    def fetch(self):
        lab, sec, act = np.zeros(self.B, np.uint8), np.zeros(self.V, np.uint8), np.zeros(self.V, np.uint8)
        lib().oracle_dpg_fetch(self.handle, _p(lab, C.c_uint8), _p(sec, C.c_uint8), _p(act, C.c_uint8))
        return lab, sec, act

    def load(self, labels=None, sector_active=None, node_active=None):
        a = [None if x is None else np.ascontiguousarray(x, np.uint8) for x in (labels, sector_active, node_active)]
        lib().oracle_dpg_load(self.handle, *[_p(x, C.c_uint8) for x in a])

    def active_dynamic_points(self, n_nodes, est):
        e = _f32(est).reshape(-1, 3)
        counts = np.zeros(4, np.int64)
        n = lib().oracle_active_dynamic_points(self.handle, n_nodes, _p(e, C.c_float), None, 0, _p(counts, C.c_int64))
        out = np.zeros((max(n, 1), 2), np.float32)
        lib().oracle_active_dynamic_points(self.handle, n_nodes, _p(e, C.c_float), _p(out, C.c_float), n,
                                           _p(counts, C.c_int64))
        names = ("active_static", "active_added", "dynamic_removed", "dynamic_added")
        res, k = {}, 0
        for name, c in zip(names, counts):
            res[name] = out[k:k + c].copy()
            k += int(c)
        return res


def retract(X, d):
    """Pose2 retraction X (+) d, ChartAtOrigin (dpg_oracle.c retract, GTSAM Values::retract)."""
    X = np.asarray(X, np.float64).reshape(-1, 3)
    d = np.asarray(d, np.float64).reshape(-1, 3)
    c, s = np.cos(X[:, 2]), np.sin(X[:, 2])
    cd, sd = np.cos(d[:, 2]), np.sin(d[:, 2])
    out = np.empty_like(X)
    out[:, 0] = X[:, 0] + (c * d[:, 0] - s * d[:, 1])
    out[:, 1] = X[:, 1] + (s * d[:, 0] + c * d[:, 1])
    out[:, 2] = np.arctan2(s * cd + c * sd, c * cd - s * sd)
    return out


class OracleIncGraph:
    """CPU restatement of the incremental per-node solve (dpg_inc.hip; optimizeGraph per node,
    dpg_slam.cc:255-329, isam_->update at :320 with ISAM2's defaults):
      isam2 -- linearization points theta; on updates whose count (this update included) is a
               multiple of relinearize_skip -- updates 10, 20, ...: GTSAM 4.0's ISAM2::update
               increments update_count_ before relinarizationNeeded(update_count_) -- variables
               with max |delta| >= relinearize_threshold take theta (+) delta; then every factor is linearized at theta, H delta = -g is solved
               (block-sparse Cholesky, oracle_gn_delta) and the estimate is theta (+) delta;
      batch -- Gauss-Newton to convergence from the current estimates (oracle_optimize_graph).
    duplicate_factors reproduces SURVEY Q1 (information x number of updates a factor has been in)."""

    def __init__(self, mode="isam2", relinearize_skip=10, relinearize_threshold=0.1, duplicate_factors=False,
                 gn_params=None):
        from dpgslam import _abi
        self._abi = _abi
        self.mode = mode
        self.skip = int(relinearize_skip)
        self.thr = float(relinearize_threshold)
        self.dup = bool(duplicate_factors)
        self.gn_params = gn_params
        self.reset()

    def reset(self):
        self.updates = 0
        self.F = np.zeros(0, self._abi.FACTOR_DTYPE)
        self.created = np.zeros(0, np.int64)
        self.theta = np.zeros((0, 3))
        self.est = np.zeros((0, 3))
        self.maxd = np.zeros(0)

    @property
    def V(self):
        return len(self.est)

    def update(self, init, factors):
        init = np.asarray(init, np.float64).reshape(-1, 3)
        V0 = self.V
        relin = self.mode == "isam2" and (self.updates + 1) % self.skip == 0 and V0 > 0
        self.updates += 1
        if relin:
            sel = self.maxd >= self.thr
            self.theta[sel] = self.est[sel]
        self.theta = np.concatenate([self.theta, init])
        self.est = np.concatenate([self.est, init])
        self.maxd = np.concatenate([self.maxd, np.zeros(len(init))])
        f = np.asarray(factors, self._abi.FACTOR_DTYPE).reshape(-1)
        self.F = np.concatenate([self.F, f])
        self.created = np.concatenate([self.created, np.full(len(f), self.updates, np.int64)])
        F = self.F.copy()
        if self.dup:
            F["info"] *= (self.updates - self.created + 1).astype(np.float64)[:, None]
        if self.mode == "isam2":
            d, err = gn_delta(self.theta, F)
            self.est = retract(self.theta, d)
            self.maxd = np.abs(d).max(1)
            return err
        X, st = optimize_graph(self.est, F, self.gn_params)
        self.est = X.copy()
        self.theta = X.copy()
        return st.final_error

    def poses(self):
        return self.est.copy()

    def load_state(self, st):
        """Take over another graph's state (api.IncGraph.export_state: the GPU graph's update count,
        factors with their creating update, theta, estimate, max |delta|) -- the lockstep tests run
        the next update from exactly the GPU's state."""
        self.updates = int(st["updates"])
        self.F = np.asarray(st["factors"], self._abi.FACTOR_DTYPE).copy()
        self.created = np.asarray(st["created"], np.int64).copy()
        self.theta = np.asarray(st["theta"], np.float64).reshape(-1, 3).copy()
        self.est = np.asarray(st["est"], np.float64).reshape(-1, 3).copy()
        self.maxd = np.asarray(st["maxd"], np.float64).copy()
