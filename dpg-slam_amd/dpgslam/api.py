"""Python mirror of the reference's hot-path interface, over the C ABI (libdpg.so).

Reference interface (file:line)                         this module
------------------------------------------------------  ---------------------------------------
calculate_ICP_COV(data_pi, model_qi, T, ICP_COV, vx,     calculate_ICP_COV(data, model, T, vx, vy,
  vy, vth)  src/icp_cov/cov_func_point_to_point.h:24        vth) -> (ICP_COV, hessian block)
DpgSLAM::runIcp(node_1, node_2, icp_results) -> bool     Context.run_icp(node_1, node_2, params)
  src/dpg_slam/dpg_slam.cc:362-446                          -> (converged, ((x, y), theta), cov)
DpgSLAM::optimizeGraph(init_estimates)                   Context.optimize_graph(poses, factors)
  src/dpg_slam/dpg_slam.cc:316-329
batched runIcp calls of reoptimize (dpg_slam.cc:85-106)  Context.upload_scans / icp_batch
"""
from __future__ import annotations

import ctypes as C
import os
import weakref
from dataclasses import dataclass

import numpy as np

from . import _abi
from ._abi import (FACTOR_DTYPE, RESULT_DTYPE, F32P, F64P, I32P, I64P, check, lib, ptr, vptr)


@dataclass
class Node:
    """The part of DpgNode (src/dpg_slam/dpg_node.h:30-36) the hot path reads: the estimated pose
    and the cached base_link cloud (getCachedPointCloudFromNode, dpg_node.cc:8-25)."""

    pose: np.ndarray   # float32 (x, y, theta)
    cloud: np.ndarray  # float32 [n, 2]


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def _f64(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64))


# ------------------------------------------------------------------------- host helpers (R1-R3)
def scan_to_cloud(ranges, angle_min, angle_max, range_max, laser=(0.2, 0.0, 0.0)) -> np.ndarray:
    r = _f32(ranges)
    out = np.empty((max(r.size, 1), 2), np.float32)
    n = lib().dpg_scan_to_cloud(ptr(r, C.c_float), r.size, angle_min, angle_max, range_max,
                                laser[0], laser[1], laser[2], ptr(out, C.c_float))
    return out[:n].copy()


def scans_to_clouds(ranges, angle_min, angle_max, range_max, laser=(0.2, 0.0, 0.0)):
    r = _f32(ranges)
    V, nb = r.shape
    pts = np.empty((V * nb, 2), np.float32)
    offs = np.empty(V + 1, np.int64)
    tot = lib().dpg_scans_to_clouds(ptr(r, C.c_float), V, nb, angle_min, angle_max, range_max,
                                    laser[0], laser[1], laser[2], ptr(pts, C.c_float), ptr(offs, C.c_int64))
    return pts[:tot].copy(), offs


def downsample(cloud, ratio: int) -> np.ndarray:
    c = _f32(cloud)
    out = np.empty((max(len(c), 1), 2), np.float32)
    n = lib().dpg_downsample_cloud(ptr(c, C.c_float), len(c), ratio, ptr(out, C.c_float))
    return out[:n].copy()


def inverse_transform_point(a, b) -> np.ndarray:
    a, b, o = _f32(a), _f32(b), np.empty(3, np.float32)
    lib().dpg_inverse_transform_point(ptr(a, C.c_float), ptr(b, C.c_float), ptr(o, C.c_float))
    return o


def transform_point(p, frame) -> np.ndarray:
    p, f, o = _f32(p), _f32(frame), np.empty(3, np.float32)
    lib().dpg_transform_point(ptr(p, C.c_float), ptr(f, C.c_float), ptr(o, C.c_float))
    return o


def icp_guess(pose_src, pose_tgt) -> np.ndarray:
    a, b, o = _f32(pose_src), _f32(pose_tgt), np.empty(6, np.float32)
    lib().dpg_icp_guess(ptr(a, C.c_float), ptr(b, C.c_float), ptr(o, C.c_float))
    return o


def odometry_factor(odom_prev, odom_cur, i_prev, i_cur, motion=(0.4, 0.4, 0.4, 0.4)):
    a, b = _f32(odom_prev), _f32(odom_cur)
    f = _abi.Factor()
    rc = lib().dpg_odometry_factor(ptr(a, C.c_float), ptr(b, C.c_float), i_prev, i_cur, *motion, C.byref(f))
    check(rc, "dpg_odometry_factor")
    return f


def odometry_factors(odom: np.ndarray, i_prev, i_cur, motion=(0.4, 0.4, 0.4, 0.4)) -> np.ndarray:
    """odometry_factor for n pairs in one call (dpg_odometry_factors): factor k between odom[i_prev[k]]
    and odom[i_cur[k]] (odom [n_odom, 3] float32); the same factors as n odometry_factor calls."""
    o = _f32(odom).reshape(-1, 3)
    a = np.ascontiguousarray(i_prev, np.int32)
    b = np.ascontiguousarray(i_cur, np.int32)
    out = np.zeros(len(a), FACTOR_DTYPE)
    if len(a):
        check(lib().dpg_odometry_factors(ptr(o, C.c_float), len(o), ptr(a, C.c_int32), ptr(b, C.c_int32), len(a),
                                         *motion, vptr(out)), "dpg_odometry_factors")
    return out


def prior_factors(nodes, sigmas=(0.2, 0.2, 0.15)) -> np.ndarray:
    """prior_factor(node, (0, 0, 0), sigmas) for every node of `nodes`."""
    n = np.asarray(nodes, np.int32).reshape(-1)
    f = np.zeros(len(n), FACTOR_DTYPE)
    f["kind"] = _abi.DPG_FACTOR_PRIOR
    f["i"] = n
    s = np.asarray(sigmas, np.float32).astype(np.float64)
    f["info"] = 1.0 / (s * s)
    return f


def prior_factor(node: int, pose=(0.0, 0.0, 0.0), sigmas=(0.2, 0.2, 0.15)) -> np.ndarray:
    """PriorFactor<Pose2> with Diagonal::Sigmas (dpg_slam.cc:44-49); sigmas are the float
    parameters new_pass_{x,y,theta}_std_dev_ (parameters.h:264-274) widened to double."""
    f = np.zeros(1, FACTOR_DTYPE)
    f["kind"] = _abi.DPG_FACTOR_PRIOR
    f["i"] = node
    f["z"] = pose
    s = np.asarray(sigmas, np.float32).astype(np.float64)
    f["info"] = 1.0 / (s * s)
    return f


def between_factor(i, j, z, sigmas=None, info=None) -> np.ndarray:
    f = np.zeros(1, FACTOR_DTYPE)
    f["kind"] = _abi.DPG_FACTOR_BETWEEN
    f["i"], f["j"], f["z"] = i, j, z
    if info is None:
        s = np.asarray(sigmas, np.float64)
        info = 1.0 / (s * s)
    f["info"] = info
    return f


def calculate_ICP_COV(data_pi, model_qi, transform, laser_x_variance=0.5, laser_y_variance=0.5,
                      laser_theta_variance=0.3, ctx: "Context | None" = None, with_hessian=True):
    """calculate_ICP_COV (cov_func_point_to_point.h:24): returns (ICP_COV 3x3, [x,y,yaw] Hessian
    block or None).  transform: 4x4 (row-major) homogeneous matrix."""
    d, m = _f32(data_pi).reshape(-1, 2), _f32(model_qi).reshape(-1, 2)
    T = _f32(transform).reshape(4, 4)
    cov = np.zeros(9, np.float64)
    hess = np.zeros(9, np.float64) if with_hessian else None
    rc = lib().icp_cov_calculate(ctx.handle if ctx else None, ptr(d, C.c_float), len(d), ptr(m, C.c_float),
                                 len(m), ptr(T, C.c_float), laser_x_variance, laser_y_variance,
                                 laser_theta_variance, ptr(cov, C.c_double), ptr(hess, C.c_double))
    check(rc, "icp_cov_calculate")
    return cov.reshape(3, 3), (hess.reshape(3, 3) if hess is not None else None)


def icp_cov_sandwich(data_pi, model_qi, transform, ctx: "Context | None" = None):
    """The 6x6 ICP covariance the reference computes and discards (cov :553-566, optional):
    (cov6 [6, 6] in x y z yaw pitch roll order, cov3 = its [x, y, yaw] block)."""
    d, m = _f32(data_pi).reshape(-1, 2), _f32(model_qi).reshape(-1, 2)
    T = _f32(transform).reshape(4, 4)
    cov6, cov3 = np.zeros(36, np.float64), np.zeros(9, np.float64)
    check(lib().icp_cov_sandwich(ctx.handle if ctx else None, ptr(d, C.c_float), len(d), ptr(m, C.c_float), len(m),
                                 ptr(T, C.c_float), ptr(cov6, C.c_double), ptr(cov3, C.c_double)), "icp_cov_sandwich")
    return cov6.reshape(6, 6), cov3.reshape(3, 3)


def results_array(n: int) -> np.ndarray:
    return np.zeros(n, RESULT_DTYPE)


def shard_plan(n_edges: int, world: int, cost=None):
    """dpg_shard_plan (host only): (owner[e], dispatch order, counts per rank) of the multi-device
    forms -- LPT over `cost` when given, else e mod world."""
    owner = np.zeros(max(n_edges, 1), np.int32)
    disp = np.zeros(max(n_edges, 1), np.int64)
    counts = np.zeros(world, np.int64)
    c = None if cost is None else _f32(cost)
    check(lib().dpg_shard_plan(ptr(c, C.c_float) if c is not None else None, n_edges, world, ptr(owner, C.c_int32),
                               ptr(disp, C.c_int64), ptr(counts, C.c_int64)), "dpg_shard_plan")
    return owner[:n_edges], disp[:n_edges], counts


def shard_reassemble(owner: np.ndarray, world: int, slice_: int, gathered: np.ndarray, rec_bytes: int) -> np.ndarray:
    """dpg_shard_reassemble (host only): the rank form's gathered slices back in the caller's order."""
    owner = np.ascontiguousarray(owner, np.int32)
    g = np.ascontiguousarray(gathered).view(np.uint8)
    out = np.zeros(len(owner) * rec_bytes, np.uint8)
    check(lib().dpg_shard_reassemble(ptr(owner, C.c_int32), len(owner), world, slice_, rec_bytes, vptr(g), vptr(out)),
          "dpg_shard_reassemble")
    return out


# ------------------------------------------------------------------------- GPU context
NCCL_ID_BYTES = 128


def nccl_unique_id() -> bytes:
    """dpg_nccl_unique_id: the id rank 0 of a one-process-per-GPU job hands to every rank."""
    buf = C.create_string_buffer(NCCL_ID_BYTES)
    check(lib().dpg_nccl_unique_id(C.cast(buf, C.c_void_p)), "dpg_nccl_unique_id")
    return buf.raw


class Context:
    """One dpg_ctx (one GPU, one HIP stream).  Creating it without a usable GPU raises."""

    def __init__(self, device: int = 0, n_gpus: int | None = None, virtual: int | None = None,
                 rank: tuple | None = None, rank_ops: tuple | None = None):
        """n_gpus: a multi-GPU context over devices device .. device + n_gpus - 1
        (dpg_ctx_create_multi: one process, RCCL between the devices); virtual=k: k contexts on
        `device` sharing one stream, the all-reduce a device-side sum (dpg_ctx_create_virtual: the
        sharded paths on one card); rank=(nccl_id bytes, rank, world): this process's device as one
        rank of a one-process-per-GPU job (dpg_ctx_create_rank); rank_ops=(collective, rank, world):
        the same over the caller's host collectives (dpg_ctx_create_rank_ops, e.g.
        dist.HostCollective over gloo); none of them: one device."""
        self._coll = None
        if virtual is not None:
            self.handle = lib().dpg_ctx_create_virtual(int(virtual), device)
        elif rank_ops is not None:
            coll, r, w = rank_ops
            self._coll = coll   # its callbacks must outlive the context
            self.handle = lib().dpg_ctx_create_rank_ops(device, C.byref(coll.ops), int(r), int(w))
        elif rank is not None:
            nid, r, w = rank
            buf = C.create_string_buffer(bytes(nid), NCCL_ID_BYTES)
            self.handle = lib().dpg_ctx_create_rank(device, C.cast(buf, C.c_void_p), int(r), int(w))
        elif n_gpus is None:
            self.handle = lib().dpg_ctx_create(device)
        else:
            devs = np.arange(device, device + int(n_gpus), dtype=np.int32)
            self.handle = lib().dpg_ctx_create_multi(int(n_gpus), ptr(devs, C.c_int32))
        if not self.handle:
            raise _abi.DpgError("dpg_ctx_create failed: " + (lib().dpg_last_error() or b"").decode())
        self.device = device
        self.n_gpus = int(lib().dpg_ctx_num_gpus(self.handle))
        self.n_ranks = int(lib().dpg_ctx_num_ranks(self.handle))
        self.rank = int(lib().dpg_ctx_rank(self.handle))
        self.n_edges = 0
        self.V = 0
        self._children = weakref.WeakSet()   # DpgStore / IncGraph objects living on this context

    def close(self):
        """Destroys the context; the DPG stores and incremental graphs created on it are closed
        first (their device state belongs to the context)."""
        if self.handle:
            for ch in list(getattr(self, "_children", ())):
                ch.close()
            lib().dpg_ctx_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_handle: int):
        check(lib().dpg_ctx_set_stream(self.handle, C.c_void_p(stream_handle)), "dpg_ctx_set_stream")

    def synchronize(self):
        check(lib().dpg_ctx_synchronize(self.handle), "dpg_ctx_synchronize")

    def set_icp_variant(self, variant: str):
        """'angular' (default), 'kdtree' or 'grid' -- nearest-neighbour machinery; results are identical."""
        v = {"angular": 3, "kdtree": 2, "grid": 1}[variant]
        check(lib().dpg_ctx_set_icp_variant(self.handle, v), "dpg_ctx_set_icp_variant")

    def set_icp_defer_cap(self, cap: int):
        """Angular ICP: windows of more than `cap` candidates are scanned by a whole wave (0: never);
        results are identical for every value."""
        check(lib().dpg_ctx_set_icp_defer_cap(self.handle, int(cap)), "dpg_ctx_set_icp_defer_cap")

    def set_cov_workgroups(self, n: int):
        """dpg_ctx_set_cov_workgroups: the covariance beside the pose graph on at most n workgroups
        (0: one per edge); results are identical for every n."""
        check(lib().dpg_ctx_set_cov_workgroups(self.handle, int(n)), "dpg_ctx_set_cov_workgroups")

    def set_solver_options(self, **kw):
        """dpg_ctx_set_solver_options: the defaults with the given fields changed (order: "auto", "md",
        "nd" or the DPG_ORDER_* value); taken by the next graph set up on this context."""
        o = _abi.default_solver_options()
        for k, v in kw.items():
            if k == "order" and isinstance(v, str):
                v = {"auto": 0, "md": 1, "nd": 2}[v]
            setattr(o, k, v)
        check(lib().dpg_ctx_set_solver_options(self.handle, C.byref(o)), "dpg_ctx_set_solver_options")

    def set_icp_schedule(self, schedule: str):
        """'measured' (default): once every edge of the staged batch has a measured cost, LPT over the
        ranks + longest-first dispatch; 'caller': e mod ranks in the caller's order.  Same results."""
        v = {"caller": 0, "measured": 1}[schedule]
        check(lib().dpg_ctx_set_icp_schedule(self.handle, v), "dpg_ctx_set_icp_schedule")

    def set_icp_kernel_variant(self, v: int):
        """Diagnostic A/B: the angular kernel's form (0 = default); results must be byte-identical."""
        check(lib().dpg_ctx_set_icp_kernel_variant(self.handle, int(v)), "dpg_ctx_set_icp_kernel_variant")

    def kdtree_build_ms(self) -> float:
        return float(lib().dpg_kdtree_build_ms(self.handle))

    # ---- runIcp ----
    def run_icp(self, node_1: Node, node_2: Node, params=None, with_hessian=False):
        """DpgSLAM::runIcp(node_1, node_2, icp_results): node_1 = target, node_2 = source.
        Returns (converged, ((tx, ty), theta), ICP_COV, result, hessian_block)."""
        p = params or _abi.default_icp_params()
        s, t = _f32(node_2.cloud).reshape(-1, 2), _f32(node_1.cloud).reshape(-1, 2)
        ps, pt = _f32(node_2.pose), _f32(node_1.pose)
        res = _abi.IcpResult()
        cov = np.zeros(9, np.float64)
        hess = np.zeros(9, np.float64) if with_hessian else None
        rc = lib().dpg_run_icp(self.handle, ptr(s, C.c_float), len(s), ptr(t, C.c_float), len(t),
                               ptr(ps, C.c_float), ptr(pt, C.c_float), C.byref(p), C.byref(res),
                               ptr(cov, C.c_double), ptr(hess, C.c_double))
        check(rc, "dpg_run_icp")
        ok = bool(res.converged) and res.status == _abi.DPG_ICP_OK
        z = ((float(res.z[0]), float(res.z[1])), float(res.z[2]))
        return ok, z, cov.reshape(3, 3), res, (hess.reshape(3, 3) if hess is not None else None)

    # ---- batched ICP ----
    def upload_scans(self, pts: np.ndarray, offsets: np.ndarray, ratio: int = 5):
        pts, offs = _f32(pts).reshape(-1, 2), np.ascontiguousarray(offsets, np.int64)
        check(lib().dpg_scans_upload(self.handle, ptr(pts, C.c_float), ptr(offs, C.c_int64), len(offs) - 1,
                                     ratio), "dpg_scans_upload")
        self.V = len(offs) - 1

    def icp_prepare(self, edges: np.ndarray, poses: np.ndarray, params=None):
        p = params or _abi.default_icp_params()
        e = np.ascontiguousarray(edges, np.int32).reshape(-1, 2)
        ps = _f32(poses).reshape(-1, 3)
        check(lib().dpg_icp_batch_prepare(self.handle, ptr(e, C.c_int32), len(e), ptr(ps, C.c_float), C.byref(p)),
              "dpg_icp_batch_prepare")
        self.n_edges = len(e)

    def icp_run(self, compute_cov=True, trace_iters=0):
        check(lib().dpg_icp_batch_run(self.handle, int(compute_cov), int(trace_iters)), "dpg_icp_batch_run")

    def icp_fetch(self, with_hessian=True):
        """Results of the staged batch, whichever call staged it (its size from dpg_icp_batch_size:
        dpg_add_node and the sweeps stage batches inside the C calls)."""
        n = int(lib().dpg_icp_batch_size(self.handle))
        if n < 0:
            check(n, "dpg_icp_batch_size")
        self.n_edges = n
        res = results_array(n)
        hess = np.zeros((n, 9), np.float64) if with_hessian else None
        check(lib().dpg_icp_batch_fetch(self.handle, vptr(res), ptr(hess, C.c_double), n), "dpg_icp_batch_fetch")
        return res, (hess.reshape(-1, 3, 3) if hess is not None else None)

    def icp_fetch_trace(self, iters: int) -> np.ndarray:
        ms = C.c_int64(0)
        check(lib().dpg_icp_batch_fetch_trace(self.handle, None, 0, C.byref(ms)), "trace size")
        tr = np.empty((self.n_edges, iters, ms.value), np.int32)
        check(lib().dpg_icp_batch_fetch_trace(self.handle, ptr(tr, C.c_int32), tr.size, C.byref(ms)), "trace fetch")
        return tr

    def icp_batch(self, edges, poses, params=None, compute_cov=True, trace_iters=0):
        self.icp_prepare(edges, poses, params)
        self.icp_run(compute_cov, trace_iters)
        return self.icp_fetch(compute_cov)

    def icp_kernel_ms(self) -> float:
        return float(lib().dpg_icp_batch_kernel_ms(self.handle))

    def cov_kernel_ms(self) -> float:
        return float(lib().dpg_cov_batch_kernel_ms(self.handle))

    def cov_overlapped(self) -> bool:
        """The last batch's covariance ran beside the pose graph (its own stream)."""
        return bool(lib().dpg_cov_batch_overlapped(self.handle))

    def icp_algorithmic_bytes(self) -> float:
        return float(lib().dpg_icp_batch_algorithmic_bytes(self.handle))

    # ---- optimizeGraph ----
    def optimize_graph(self, poses: np.ndarray, factors: np.ndarray, params=None):
        """Batch Gauss-Newton to convergence; returns (poses [V,3] float64, stats)."""
        X = _f64(poses).reshape(-1, 3).copy()
        F = np.ascontiguousarray(factors, FACTOR_DTYPE)
        gp = params or _abi.default_gn_params()
        st = _abi.GnStats()
        check(lib().dpg_optimize_graph(self.handle, ptr(X, C.c_double), len(X), vptr(F), len(F), C.byref(gp),
                                       C.byref(st)), "dpg_optimize_graph")
        return X, st

    # ---- sharded GN step API ----
    def gn_setup(self, V: int, factors: np.ndarray, shard=(0, None), params=None):
        F = np.ascontiguousarray(factors, FACTOR_DTYPE)
        b, e = shard[0], (len(F) if shard[1] is None else shard[1])
        gp = params or _abi.default_gn_params()
        check(lib().dpg_gn_setup(self.handle, V, vptr(F), len(F), b, e, C.byref(gp)), "dpg_gn_setup")
        return int(lib().dpg_gn_hb_size(self.handle))

    def gn_take_icp(self, first: int, count: int, n_always: int, params=None):
        p = params or _abi.default_icp_params()
        check(lib().dpg_gn_take_icp_measurements(self.handle, first, count, n_always, C.byref(p)),
              "dpg_gn_take_icp_measurements")

    def gn_set_poses(self, poses):
        X = _f64(poses).reshape(-1, 3)
        check(lib().dpg_gn_set_poses(self.handle, ptr(X, C.c_double)), "dpg_gn_set_poses")

    def gn_setup_profile(self) -> dict:
        """dpg_gn_setup_profile: host ms of the last gn_setup's parts."""
        out = np.zeros(5, np.float64)
        check(lib().dpg_gn_setup_profile(self.handle, ptr(out, C.c_double)), "dpg_gn_setup_profile")
        return dict(zip(("pattern_lists_bsr", "chol_symbolic", "chol_plan", "wait_alloc_upload", "chol_upload"),
                        (float(x) for x in out)))

    def gn_run(self, V: int | None = None):
        """The whole GN loop natively (dpg_gn_run) from the poses of gn_set_poses; returns
        (stats dict, poses [V, 3] or None when V is None)."""
        X = np.empty((V, 3), np.float64) if V else None
        st = _abi.GnStats()
        check(lib().dpg_gn_run(self.handle, ptr(X, C.c_double) if X is not None else None, C.byref(st)),
              "dpg_gn_run")
        return {k: getattr(st, k) for k, _ in _abi.GnStats._fields_}, X

    def gn_get_poses(self, V: int) -> np.ndarray:
        X = np.empty((V, 3), np.float64)
        check(lib().dpg_gn_get_poses(self.handle, ptr(X, C.c_double)), "dpg_gn_get_poses")
        return X

    def gn_assemble(self, hb_dev_ptr: int | None = None):
        check(lib().dpg_gn_assemble(self.handle, C.c_void_p(hb_dev_ptr) if hb_dev_ptr else None), "dpg_gn_assemble")

    def gn_solve_retract(self, hb_dev_ptr: int | None = None):
        d, e, it = C.c_double(0), C.c_double(0), C.c_int32(0)
        check(lib().dpg_gn_solve_retract(self.handle, C.c_void_p(hb_dev_ptr) if hb_dev_ptr else None, C.byref(d),
                                         C.byref(e), C.byref(it)), "dpg_gn_solve_retract")
        return d.value, e.value, it.value

    def gn_solve_retract_async(self, hb_dev_ptr: int | None = None):
        check(lib().dpg_gn_solve_retract_async(self.handle, C.c_void_p(hb_dev_ptr) if hb_dev_ptr else None),
              "dpg_gn_solve_retract_async")

    def gn_fetch(self, hb_dev_ptr: int | None = None):
        out = np.zeros(3, np.float64)
        check(lib().dpg_gn_fetch(self.handle, C.c_void_p(hb_dev_ptr) if hb_dev_ptr else None, ptr(out, C.c_double)),
              "dpg_gn_fetch")
        return float(out[0]), float(out[1]), int(out[2])

    def gn_factorizations(self) -> int:
        return int(lib().dpg_gn_factorizations(self.handle))

    def loop_closure_candidates(self, est: np.ndarray, passes: np.ndarray, within: float = 5.0,
                                across: float = 2.0) -> np.ndarray:
        """reoptimize's candidate pairs (j, i) on the GPU (dpg_slam.cc:91-98), reference order."""
        e, ps = _f32(est).reshape(-1, 3), np.ascontiguousarray(passes, np.int32)
        L = lib()
        n = L.dpg_loop_closure_candidates(self.handle, len(e), ptr(ps, C.c_int32), ptr(e, C.c_float), within, across,
                                          None, 0)
        if n < 0:
            check(int(n), "dpg_loop_closure_candidates")
        out = np.zeros((max(n, 1), 2), np.int32)
        n2 = L.dpg_loop_closure_candidates(self.handle, len(e), ptr(ps, C.c_int32), ptr(e, C.c_float), within, across,
                                           ptr(out, C.c_int32), n)
        if n2 < 0:
            check(int(n2), "dpg_loop_closure_candidates")
        return out[:n]

    def get_map(self, est: np.ndarray, display_points_fraction: int = 10) -> np.ndarray:
        """DpgSLAM::GetMap (dpg_slam.cc:555-575) over the uploaded clouds: map-frame points [K, 2]."""
        e = _f32(est).reshape(-1, 3)
        L = lib()
        n = L.dpg_get_map(self.handle, ptr(e, C.c_float), display_points_fraction, None, 0)
        if n < 0:
            check(int(n), "dpg_get_map")
        out = np.zeros((max(n, 1), 2), np.float32)
        n2 = L.dpg_get_map(self.handle, ptr(e, C.c_float), display_points_fraction, ptr(out, C.c_float), n)
        if n2 < 0:
            check(int(n2), "dpg_get_map")
        return out[:n]

    def get_map_kernel_ms(self) -> float:
        return float(lib().dpg_get_map_kernel_ms(self.handle))

    def reoptimize(self, passes: np.ndarray, est: np.ndarray, odom: np.ndarray, icp_params=None, gn_params=None,
                   reopt_params=None):
        """DpgSLAM::reoptimize (dpg_slam.cc:35-120) over the uploaded scans: candidate search, one
        batched ICP of every edge, factors, batch GN.  Returns (poses [V,3] f64, ReoptStats)."""
        e, o = _f32(est).reshape(-1, 3), _f32(odom).reshape(-1, 3)
        ps = np.ascontiguousarray(passes, np.int32)
        ip = icp_params or _abi.default_icp_params()
        gp = gn_params or _abi.default_gn_params()
        rp = reopt_params or _abi.default_reopt_params()
        X = np.zeros((len(e), 3), np.float64)
        st = _abi.ReoptStats()
        check(lib().dpg_reoptimize(self.handle, len(e), ptr(ps, C.c_int32), ptr(e, C.c_float), ptr(o, C.c_float),
                                   C.byref(ip), C.byref(gp), C.byref(rp), ptr(X, C.c_double), C.byref(st)),
              "dpg_reoptimize")
        self.n_edges = int(st.n_icp_edges)   # the sweep's batch stays staged: icp_fetch returns its results
        return X, st

    def gn_times_ms(self):
        return float(lib().dpg_gn_last_assemble_ms(self.handle)), float(lib().dpg_gn_last_solve_ms(self.handle))


# ------------------------------------------------------------------ DPG change detection
def _ctx_gone(child) -> bool:
    """The context a DpgStore / IncGraph lives on is already destroyed.  Context.close closes its
    children first, but when both sit in one reference cycle the garbage collector clears the
    context's weak child set before any finalizer runs, and may finalize the context first.
    dpg_ctx_destroy has then already destroyed the child (a context destroys the incremental graphs
    and DPG stores created on it: device buffers, pinned mirrors, events, helper thread), so the
    handle is dangling and only dropped here."""
    ctx = getattr(child, "ctx", None)
    return ctx is not None and getattr(ctx, "handle", None) is None


class DpgStore:
    """The dynamic node state of DpgSLAM (per-beam labels and sectors, per-node sector activation and
    activity, dpg_measurement.h / dpg_node.h), resident on the context's GPU, and executeDPG over it
    (dpg_slam.cc:865-886).  ranges: [V, n_beams] (or concatenated with offsets); geom: [V, 3] =
    angle_min, angle_max, range_max per scan."""

    def __init__(self, ctx: Context, ranges, geom, offsets=None, params=None):
        r = _f32(ranges)
        if offsets is None:
            V, nb = r.shape
            offsets = np.arange(V + 1, dtype=np.int64) * nb
        off = np.ascontiguousarray(offsets, np.int64)
        self.V = len(off) - 1
        self.B = int(off[-1])
        g = _f32(geom).reshape(self.V, 3)
        self.params = params or _abi.default_change_params()
        self.ctx = ctx
        self.handle = lib().dpg_dpg_create(ctx.handle, self.V, ptr(off, C.c_int64), ptr(r.reshape(-1), C.c_float),
                                           ptr(g, C.c_float), C.byref(self.params))
        if not self.handle:
            raise _abi.DpgError("dpg_dpg_create failed: " + (lib().dpg_last_error() or b"").decode())
        ctx._children.add(self)

    def close(self):
        if getattr(self, "handle", None):
            if _ctx_gone(self):   # finalized after its context: dpg_ctx_destroy already destroyed it
                self.handle = None
                return
            lib().dpg_dpg_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def append(self, ranges, geom, offsets=None):
        """Add nodes' scans at the end (dpg_dpg_append); the existing node state is kept."""
        r = _f32(ranges)
        if offsets is None:
            n, nb = r.shape
            offsets = np.arange(n + 1, dtype=np.int64) * nb
        off = np.ascontiguousarray(offsets, np.int64)
        g = _f32(geom).reshape(-1, 3)
        check(lib().dpg_dpg_append(self.handle, len(off) - 1, ptr(off, C.c_int64), ptr(r.reshape(-1), C.c_float),
                                   ptr(g, C.c_float)), "dpg_dpg_append")
        self.V += len(off) - 1
        self.B += int(off[-1] - off[0])

    def execute_dpg(self, n_nodes: int, current_pass_len: int, est, chain_poses=None) -> "_abi.ChangeStats":
        """executeDPG (dpg_slam.cc:865-886).  chain_poses [chain_n][3]: the poses of the pose chain as the
        reference's current_pass_nodes_ copies hold them (dpg_slam.cc:195,307,598), placing the chain
        grids and the proximity search (dpg_execute_dpg_chain); None places them at est."""
        e = _f32(est).reshape(-1, 3)
        st = _abi.ChangeStats()
        if chain_poses is None:
            check(lib().dpg_execute_dpg(self.handle, n_nodes, current_pass_len, ptr(e, C.c_float), C.byref(st)),
                  "dpg_execute_dpg")
        else:
            c = _f32(chain_poses).reshape(-1, 3)
            check(lib().dpg_execute_dpg_chain(self.handle, n_nodes, current_pass_len, ptr(e, C.c_float),
                                              ptr(c, C.c_float), C.byref(st)), "dpg_execute_dpg_chain")
        return st

    def fetch(self):
        """(labels [B] u8, sector_active [V] u8 bitmask, node_active [V] u8)."""
        lab = np.zeros(self.B, np.uint8)
        sec = np.zeros(self.V, np.uint8)
        act = np.zeros(self.V, np.uint8)
        check(lib().dpg_dpg_fetch(self.handle, ptr(lab, C.c_uint8), ptr(sec, C.c_uint8), ptr(act, C.c_uint8)),
              "dpg_dpg_fetch")
        return lab, sec, act

    def load(self, labels=None, sector_active=None, node_active=None):
        a = [None if x is None else np.ascontiguousarray(x, np.uint8) for x in (labels, sector_active, node_active)]
        check(lib().dpg_dpg_load(self.handle, *[ptr(x, C.c_uint8) for x in a]), "dpg_dpg_load")

    def active_dynamic_points(self, n_nodes: int, est):
        """getActiveAndDynamicMapPoints (dpg_slam.cc:832-863): dict of the four [n, 2] point lists."""
        e = _f32(est).reshape(-1, 3)
        counts = np.zeros(4, np.int64)
        n = lib().dpg_active_dynamic_points(self.handle, n_nodes, ptr(e, C.c_float), None, 0, ptr(counts, C.c_int64))
        if n < 0:
            check(int(n), "dpg_active_dynamic_points")
        out = np.zeros((max(n, 1), 2), np.float32)
        n2 = lib().dpg_active_dynamic_points(self.handle, n_nodes, ptr(e, C.c_float), ptr(out, C.c_float), n,
                                             ptr(counts, C.c_int64))
        if n2 < 0:
            check(int(n2), "dpg_active_dynamic_points")
        names = ("active_static", "active_added", "dynamic_removed", "dynamic_added")
        res, k = {}, 0
        for name, c in zip(names, counts):
            res[name] = out[k:k + c].copy()
            k += int(c)
        return res


class IncGraph:
    """The incremental per-node pose graph (dpg_inc): isam_->update once per new node
    (dpg_slam.cc:255-329), device-resident, growing in place.  mode: "isam2" (ISAM2 defaults: partial
    relinearization, threshold 0.1, skip 10) or "batch" (Gauss-Newton to convergence per update).
    full_refactor: every ISAM2 update refactors every Cholesky front (default: only the fronts the
    update touches and their ancestors -- isam_->update's partial re-elimination, same numbers)."""

    def __init__(self, ctx: Context, mode: str = "isam2", duplicate_factors: bool = False, reorder_every: int = 32,
                 gn_params=None, full_refactor: bool = False):
        self.ctx = ctx
        p = _abi.default_inc_params()
        p.mode = {"isam2": _abi.DPG_INC_ISAM2, "batch": _abi.DPG_INC_BATCH}[mode]
        p.duplicate_factors = 1 if duplicate_factors else 0
        p.reorder_every = int(reorder_every)
        p.full_refactor = 1 if full_refactor else 0
        if gn_params is not None:
            p.gn = gn_params
        self.params = p
        self.handle = lib().dpg_inc_create(ctx.handle, C.byref(p))
        if not self.handle:
            raise _abi.DpgError("dpg_inc_create failed: " + (lib().dpg_last_error() or b"").decode())
        ctx._children.add(self)

    def close(self):
        if getattr(self, "handle", None):
            if _ctx_gone(self):   # finalized after its context: dpg_ctx_destroy already destroyed it
                self.handle = None
                return
            lib().dpg_inc_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def V(self) -> int:
        return int(lib().dpg_inc_num_nodes(self.handle))

    def reset(self):
        check(lib().dpg_inc_reset(self.handle), "dpg_inc_reset")

    def update(self, init: np.ndarray, factors: np.ndarray) -> "_abi.IncStats":
        """isam_->update(new factors, new values): init [n_new, 3] initial values of the new nodes."""
        X = np.ascontiguousarray(np.asarray(init, np.float64).reshape(-1, 3))
        F = np.ascontiguousarray(factors, FACTOR_DTYPE) if factors is not None and len(factors) else \
            np.zeros(0, FACTOR_DTYPE)
        st = _abi.IncStats()
        check(lib().dpg_inc_update(self.handle, len(X), ptr(X, C.c_double) if len(X) else None,
                                   vptr(F) if len(F) else None, len(F), C.byref(st)), "dpg_inc_update")
        return st

    def poses(self, n: int | None = None) -> np.ndarray:
        n = self.V if n is None else int(n)
        X = np.zeros((max(n, 1), 3), np.float64)
        check(lib().dpg_inc_get_poses(self.handle, ptr(X, C.c_double), n), "dpg_inc_get_poses")
        return X[:n]

    def save(self, path: str):
        """dpg_inc_save: the graph and its context's scan store to one checkpoint file."""
        check(lib().dpg_inc_save(self.handle, os.fsencode(path)), "dpg_inc_save")

    def export_state(self) -> dict:
        """dpg_inc_export: the update count, factors (+ the update that added each), linearization
        points, estimate and last max |delta| per node, as host arrays."""
        L = lib()
        n = L.dpg_inc_export(self.handle, None, None, None, 0, None, None, None)
        if n < 0:
            check(int(n), "dpg_inc_export")
        V = self.V
        upd = C.c_int64(0)
        F = np.zeros(max(n, 1), FACTOR_DTYPE)
        cr = np.zeros(max(n, 1), np.int32)
        th, es, md = np.zeros((max(V, 1), 3)), np.zeros((max(V, 1), 3)), np.zeros(max(V, 1))
        m = L.dpg_inc_export(self.handle, C.byref(upd), vptr(F), ptr(cr, C.c_int32), n, ptr(th, C.c_double),
                             ptr(es, C.c_double), ptr(md, C.c_double))
        if m < 0:
            check(int(m), "dpg_inc_export")
        return {"updates": int(upd.value), "factors": F[:n], "created": cr[:n], "theta": th[:V], "est": es[:V],
                "maxd": md[:V]}

    @classmethod
    def load(cls, ctx: Context, path: str) -> "IncGraph":
        """dpg_inc_load: a graph restored from a checkpoint on ctx (ctx's scan store is replaced)."""
        g = cls.__new__(cls)
        g.ctx = ctx
        g.params = None
        g.handle = lib().dpg_inc_load(ctx.handle if ctx is not None else None, os.fsencode(path))
        if not g.handle:
            raise _abi.DpgError("dpg_inc_load failed: " + (lib().dpg_last_error() or b"").decode())
        if ctx is not None:
            ctx._children.add(g)
        return g

    def add_node(self, cloud, passes, init_pose, extra=None, icp_params=None, reopt_params=None,
                 non_successive=True) -> "_abi.AddNodeStats":
        """dpg_add_node: the node's cloud joins the device scan store, its successive + loop-closure
        alignments run as ONE batched ICP, and the factors (+ extra: pass prior / odometry) go into
        one update.  passes: pass number of every node, the new one last."""
        cl = _f32(cloud).reshape(-1, 2)
        ps = np.ascontiguousarray(passes, np.int32)
        ip = _f32(init_pose).reshape(3)
        E = np.ascontiguousarray(extra, FACTOR_DTYPE) if extra is not None and len(extra) else np.zeros(0, FACTOR_DTYPE)
        st = _abi.AddNodeStats()
        check(lib().dpg_add_node(self.handle, ptr(cl, C.c_float) if len(cl) else None, len(cl), ptr(ps, C.c_int32),
                                 ptr(ip, C.c_float), vptr(E) if len(E) else None, len(E),
                                 C.byref(icp_params or _abi.default_icp_params()),
                                 C.byref(reopt_params or _abi.default_reopt_params()), 1 if non_successive else 0,
                                 C.byref(st)), "dpg_add_node")
        return st

    def reoptimize(self, passes, est, odom, icp_params=None, reopt_params=None):
        """dpg_reoptimize_inc: the reoptimize sweep on the graph's context (every node's cloud is in
        its scan store), then this graph rebuilt from the sweep's factors by one update from est
        (dpg_slam.cc:35-120).  Returns (poses [V,3] f64, ReoptStats)."""
        e, o = _f32(est).reshape(-1, 3), _f32(odom).reshape(-1, 3)
        ps = np.ascontiguousarray(passes, np.int32)
        X = np.zeros((len(e), 3), np.float64)
        st = _abi.ReoptStats()
        check(lib().dpg_reoptimize_inc(self.handle, len(e), ptr(ps, C.c_int32), ptr(e, C.c_float), ptr(o, C.c_float),
                                       C.byref(icp_params or _abi.default_icp_params()),
                                       C.byref(reopt_params or _abi.default_reopt_params()), ptr(X, C.c_double),
                                       C.byref(st)), "dpg_reoptimize_inc")
        return X, st

    def add_node_pairs(self, cloud, init_pose, pairs, extra=None, successive=True, icp_params=None) -> "_abi.AddNodeStats":
        """dpg_add_node_pairs: as add_node, with the loop-closure alignments given (pairs [k, 2] =
        (node_1 target, node_2 source), keys <= the new node's id)."""
        cl = _f32(cloud).reshape(-1, 2)
        ip = _f32(init_pose).reshape(3)
        pr = np.ascontiguousarray(np.asarray(pairs, np.int32).reshape(-1, 2))
        E = np.ascontiguousarray(extra, FACTOR_DTYPE) if extra is not None and len(extra) else np.zeros(0, FACTOR_DTYPE)
        st = _abi.AddNodeStats()
        check(lib().dpg_add_node_pairs(self.handle, ptr(cl, C.c_float) if len(cl) else None, len(cl), ptr(ip, C.c_float),
                                       vptr(E) if len(E) else None, len(E), ptr(pr, C.c_int32) if len(pr) else None,
                                       len(pr), 1 if successive else 0, C.byref(icp_params or _abi.default_icp_params()),
                                       C.byref(st)), "dpg_add_node_pairs")
        return st
