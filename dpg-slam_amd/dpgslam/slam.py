"""DpgSLAM -- the public API of dpg_slam::DpgSLAM (src/dpg_slam/dpg_slam.h:283-335) as a host-side
driver over the MI355X C ABI: the per-node pipeline the ROS glue runs (ObserveOdometry,
ObserveLaser -> updatePoseGraph -> runIcp / optimizeGraph -> executeDPG, incrementPassNumber ->
reoptimize, GetPose, GetMap, getActiveAndDynamicMapPoints).

The bookkeeping (odometry thresholds, node creation, which scans are aligned, which factors are
added) follows dpg_slam.cc line by line in float32 where the reference is float; every numeric
step runs through a backend: GpuBackend (the HIP kernels, dpgslam.api) by default, or any object
with the same methods (tests/slam_oracle.py holds the CPU restatement the tests compare against).
optimizeGraph is the incremental graph (dpg_inc): one ISAM2-semantics update per node by default
(inc_mode="isam2"), or Gauss-Newton to convergence per node (inc_mode="batch"); SURVEY Q1/Q6.
"""
from __future__ import annotations

import ctypes as C
import math

import time

import numpy as np

from . import _abi, api
from ._abi import FACTOR_DTYPE, lib

f32 = np.float32


def _angle_mod(a) -> np.float32:
    """math_utils::AngleMod<float> (math_utils.h:13-16): the subtraction in double."""
    ad = float(f32(a))
    ad -= (math.pi * 2.0) * float(np.rint(ad / (math.pi * 2.0)))
    return f32(ad)


def _icp_factor(res, i, j, p) -> np.ndarray:
    """addObservationConstraint (dpg_slam.cc:331-338) over the ICP result (dpg_icp_factor)."""
    f = _abi.Factor()
    r = _abi.IcpResult.from_buffer_copy(np.ascontiguousarray(res).tobytes()) if isinstance(res, np.ndarray) else res
    lib().dpg_icp_factor(C.byref(r), i, j, C.byref(p), C.byref(f))
    return np.frombuffer(bytes(f), FACTOR_DTYPE).copy()


class GpuBackend:
    """The numeric steps of DpgSLAM on the MI355X (dpgslam.api over the C ABI).  Per node ONE call,
    dpg_add_node: the node's cloud joins the device scan store, its successive and loop-closure
    alignments run as one batched ICP, and the factors go into the incremental graph (dpg_inc)."""

    def __init__(self, ctx: api.Context, inc_mode: str = "isam2"):
        self.ctx = ctx
        self.inc = api.IncGraph(ctx, mode=inc_mode)
        self.stored = 0        # nodes in the context's scan store (dpg_add_node appends each node's cloud)
        self.last_add = None   # AddNodeStats of the last node

    def add_node(self, cloud, passes, init_pose, extra, icp_params, reopt_params, non_successive):
        st = self.inc.add_node(cloud, passes, init_pose, extra, icp_params, reopt_params, non_successive)
        self.stored += 1
        self.last_add = st
        n_icp = (1 if len(passes) > 1 else 0) + int(st.n_loop_closures)
        return n_icp, self.inc.poses()

    def icp_batch(self, clouds, edges, est, p):
        """clouds() -> (pts, offsets) of every node; the store already holds them when every node
        came through add_node."""
        if self.stored != len(est):
            pts, offsets = clouds()
            self.ctx.upload_scans(pts, offsets, p.downsample_icp_points_ratio)
            self.stored = len(est)
        res, _ = self.ctx.icp_batch(edges, est, p, compute_cov=False)
        return res

    def candidates(self, est, passes, within, across):
        return self.ctx.loop_closure_candidates(est, passes, within, across)

    def rebuild_graph(self, est, F):
        """reoptimize's new ISAM2 + new graph and its one update (dpg_slam.cc:36-39,111-119); the
        scan store holds every node's cloud (icp_batch uploaded them)."""
        self.inc.reset()
        self.last_rebuild = self.inc.update(np.asarray(est, np.float64), F)
        return self.inc.poses()

    def store(self, ranges, geom, offsets, params):
        return api.DpgStore(self.ctx, ranges, geom, offsets=offsets, params=params)

    def get_map(self, clouds, est, fraction, ratio):
        if self.stored != len(est):
            pts, offsets = clouds()
            self.ctx.upload_scans(pts, offsets, ratio)
            self.stored = len(est)
        return self.ctx.get_map(est, fraction)


class DpgSLAM:
    """dpg_slam::DpgSLAM.  Parameters default to parameters.h (PoseGraphParameters, DpgParameters,
    VisualizationParams.display_points_fraction_)."""

    def __init__(self, backend="gpu", ctx: api.Context | None = None, icp_params=None, gn_params=None,
                 change_params=None, min_dist_between_nodes=1.0, min_angle_between_nodes=math.pi / 6.0,
                 non_successive_scan_constraints=True, odometry_constraints=True,
                 max_dist_within_pass=5.0, max_dist_across_passes=2.0, new_pass_std_dev=(0.2, 0.2, 0.15),
                 motion_model=(0.4, 0.4, 0.4, 0.4), display_points_fraction=10, inc_mode="isam2"):
        if backend == "gpu":
            self.ctx = ctx or api.Context(0)
            self.be = GpuBackend(self.ctx, inc_mode)
        elif isinstance(backend, str):
            raise ValueError(f"unknown backend {backend!r} (pass a backend object for anything but 'gpu')")
        else:
            self.be = backend
        self.icp_params = icp_params or _abi.default_icp_params()
        self.gn_params = gn_params or _abi.default_gn_params()
        self.change_params = change_params or _abi.default_change_params()
        self.laser = tuple(float(x) for x in self.change_params.laser)
        self.min_dist = f32(min_dist_between_nodes)
        self.min_angle = f32(min_angle_between_nodes)
        self.non_successive = bool(non_successive_scan_constraints)
        self.odometry_constraints = bool(odometry_constraints)
        self.within, self.across = f32(max_dist_within_pass), f32(max_dist_across_passes)
        self.prior_sigmas = tuple(new_pass_std_dev)
        self.motion = tuple(motion_model)
        self.fraction = int(display_points_fraction)
        # DpgSLAM state (dpg_slam.h private members)
        self.pass_number = 0
        self.odom_initialized = False
        self.first_scan_for_pass = True
        self.cum_dist = f32(0.0)
        self.prev_odom = np.zeros(3, f32)               # prev_odom_loc_, prev_odom_angle_
        self.odom_at_last_align = np.zeros(3, f32)      # odom_{loc,angle}_at_last_laser_align_
        self.poses = np.zeros((0, 3), f32)               # dpg_nodes_ estimated positions (float32)
        self.node_pass = np.zeros(0, np.int32)
        self.ranges: list[np.ndarray] = []
        self.geom: list[tuple] = []
        self.clouds: list[np.ndarray] = []
        self.odom_only: list[np.ndarray] = []
        self.current_pass: list[int] = []
        self.factors: list[np.ndarray] = []             # reoptimize's graph (the per-node factors live in the backend)
        self.n_factors = 0                              # graph_->size()
        self._store = None
        self._store_V = 0
        self.last_dpg = None                            # dpg_change_stats of the last executeDPG

    # ------------------------------------------------------------------ public API
    def ObserveOdometry(self, odom_loc, odom_angle):
        """dpg_slam.cc:515-526."""
        self.odom_initialized = True
        loc = np.asarray(odom_loc, f32)
        d = loc - self.prev_odom[:2]
        self.cum_dist = f32(self.cum_dist + f32(np.sqrt(f32(d[0] * d[0]) + f32(d[1] * d[1]))))
        self.prev_odom = np.array([loc[0], loc[1], f32(odom_angle)], f32)

    def ObserveLaser(self, ranges, range_min, range_max, angle_min, angle_max):
        """dpg_slam.cc:122-140."""
        if not self.odom_initialized:
            return
        if not self._update_pose_graph(np.asarray(ranges, f32), f32(range_max), f32(angle_min), f32(angle_max)):
            return
        if self.pass_number >= 1:
            self.last_dpg = self.executeDPG()

    def incrementPassNumber(self):
        """dpg_slam.cc:25-33."""
        self.pass_number += 1
        self.odom_initialized = False
        self.first_scan_for_pass = True
        self.current_pass = []
        self.reoptimize()

    def GetPose(self):
        """dpg_slam.cc:528-553: the last node's estimate plus the odometry not yet in the graph."""
        loc = self.poses[-1][:2] if len(self.poses) else np.zeros(2, f32)
        ang = self.poses[-1][2] if len(self.poses) else f32(0)
        un = self.prev_odom[:2] - self.odom_at_last_align[:2]
        dth = _angle_mod(self.prev_odom[2] - self.odom_at_last_align[2])   # AngleDiff
        disp = api.transform_point(np.array([un[0], un[1], 0], f32), np.array([0, 0, -self.odom_at_last_align[2]], f32))
        rot = api.transform_point(np.array([disp[0], disp[1], 0], f32), np.array([0, 0, ang], f32))
        return np.array([loc[0] + rot[0], loc[1] + rot[1]], f32), f32(ang + dth)

    def GetMap(self):
        """dpg_slam.cc:555-575."""
        if not len(self.poses):
            return np.zeros((0, 2), f32)
        return self.be.get_map(self._clouds, self.poses, self.fraction, self.icp_params.downsample_icp_points_ratio)

    def GetActiveAndDynamicMapPoints(self):
        """getActiveAndDynamicMapPoints (dpg_slam.cc:832-863) over the current node state."""
        return self._dpg_store().active_dynamic_points(len(self.poses), self.poses)

    def executeDPG(self):
        """dpg_slam.cc:865-886 (dpg_execute_dpg on the node store)."""
        return self._dpg_store().execute_dpg(len(self.poses), len(self.current_pass), self.poses)

    def reoptimize(self):
        """dpg_slam.cc:35-120: a fresh graph -- per node the pass prior or the odometry Between, the
        successive alignment (always a factor) and every loop-closure candidate (a factor when
        converged), all aligned in one batch from the current estimates -- then one update of a new
        graph from the current estimates."""
        V = len(self.poses)
        if V == 0:
            return
        t0 = time.perf_counter()
        est = self.poses.copy()
        passes = self.node_pass
        lc = self.be.candidates(est, passes, float(self.within), float(self.across))
        t1 = time.perf_counter()
        succ = np.stack([np.arange(V - 1), np.arange(1, V)], 1).astype(np.int32)
        edges = np.concatenate([succ, np.asarray(lc, np.int32).reshape(-1, 2)], 0)
        res = None
        if len(edges):
            res = self.be.icp_batch(self._clouds, edges, est, self.icp_params)
        t2 = time.perf_counter()
        # per node, in node order: the pass's prior on its first node, else the odometry Between
        # from the previous node (dpg_slam.cc:41-75) -- built for all nodes at once
        pv = np.asarray(passes)
        start = np.ones(V, bool)
        start[1:] = pv[1:] != pv[:-1]
        keep_n = start | bool(self.odometry_constraints)
        Fn = np.zeros(V, FACTOR_DTYPE)
        Fn[start] = api.prior_factors(np.nonzero(start)[0], sigmas=self.prior_sigmas)
        odo = np.nonzero(~start)[0] if self.odometry_constraints else np.zeros(0, np.int64)
        if len(odo):
            Fn[odo] = api.odometry_factors(np.asarray(self.odom_only, f32), odo - 1, odo, self.motion)
        F = [Fn[keep_n]]
        if len(edges):
            # addObservationConstraint per aligned pair (dpg_icp_factor, vectorised): the successive
            # pairs always, a loop closure when its alignment converged (dpg_slam.cc:85-104)
            keep = np.ones(len(edges), bool)
            keep[len(succ):] = (res["converged"][len(succ):] != 0) & (res["status"][len(succ):] == _abi.DPG_ICP_OK)
            Fi = np.zeros(int(keep.sum()), FACTOR_DTYPE)
            Fi["kind"] = _abi.DPG_FACTOR_BETWEEN
            Fi["i"], Fi["j"] = edges[keep, 0], edges[keep, 1]
            Fi["z"] = res["z"][keep].astype(np.float64)
            p = self.icp_params
            Fi["info"] = [1.0 / float(f32(p.laser_x_variance)), 1.0 / float(f32(p.laser_y_variance)),
                          1.0 / float(f32(p.laser_theta_variance))]
            F.append(Fi)
        F = np.concatenate([np.asarray(f, FACTOR_DTYPE).reshape(-1) for f in F])
        self.factors = F
        self.n_factors = len(F)
        t3 = time.perf_counter()
        X = self.be.rebuild_graph(est.astype(np.float64), F)
        self.poses = np.asarray(X, f32).reshape(-1, 3)
        # the sweep's phases (ms): candidate search, the batched ICP, the factor list, the new graph's update
        self.last_sweep_ms = {"candidates": (t1 - t0) * 1e3, "icp": (t2 - t1) * 1e3, "factors": (t3 - t2) * 1e3,
                              "update": (time.perf_counter() - t3) * 1e3, "edges": int(len(edges))}
        st = getattr(self.be, "last_rebuild", None)
        if st is not None:
            self.last_sweep_ms.update(update_symbolic=st.ms_symbolic, update_numeric=st.ms_numeric,
                                      gn_iterations=int(st.gn_iterations))

    # ------------------------------------------------------------------ internals
    def _odometry_factor(self, prev, cur, i, j):
        f = api.odometry_factor(prev, cur, i, j, self.motion)
        return np.frombuffer(bytes(f), FACTOR_DTYPE).copy()

    def _clouds(self):
        offs = np.zeros(len(self.clouds) + 1, np.int64)
        offs[1:] = np.cumsum([len(c) for c in self.clouds])
        pts = np.concatenate(self.clouds) if self.clouds else np.zeros((0, 2), f32)
        return np.ascontiguousarray(pts, f32), offs

    def _create_node(self, ranges, range_max, angle_min, angle_max, pose):
        """createNode (dpg_slam.cc:488-513): the base_link cloud of the scan, MAX_RANGE dropped."""
        cloud = api.scan_to_cloud(ranges, angle_min, angle_max, range_max, self.laser)
        self.poses = np.concatenate([self.poses, np.asarray(pose, f32).reshape(1, 3)])
        self.node_pass = np.append(self.node_pass, np.int32(self.pass_number))
        self.ranges.append(ranges.copy())
        self.geom.append((angle_min, angle_max, range_max))
        self.clouds.append(np.ascontiguousarray(cloud, f32))
        return len(self.poses) - 1

    def _should_process_laser(self):
        """dpg_slam.cc:577-589."""
        angle_diff = f32(abs(_angle_mod(self.prev_odom[2] - self.odom_at_last_align[2])))
        if self.cum_dist > self.min_dist or angle_diff > self.min_angle:
            self.cum_dist = f32(0.0)
            return True
        return False

    def _update_pose_graph(self, ranges, range_max, angle_min, angle_max):
        """dpg_slam.cc:160-253."""
        if self.first_scan_for_pass:
            self.first_scan_for_pass = False
            n = self._create_node(ranges, range_max, angle_min, angle_max, (0.0, 0.0, 0.0))
            extra = api.prior_factor(n, sigmas=self.prior_sigmas)
            self.odom_only.append(self.prev_odom.copy())
            self.odom_at_last_align = self.prev_odom.copy()
            if self.pass_number == 0:   # the first node: the prior only, then optimizeGraph (:189-202)
                self._add_node(n, extra, aligned=False)
                return False
            self._add_node(n, extra)
            return True
        if not self._should_process_laser():
            return False
        rel = api.inverse_transform_point(self.prev_odom, self.odom_at_last_align)   # displacement since the last node
        pose = api.transform_point(rel, self.poses[-1])                                # createRelativePositionedNode
        n = self._create_node(ranges, range_max, angle_min, angle_max, pose)
        extra = self._odometry_factor(self.odom_at_last_align, self.prev_odom, n - 1, n) if self.odometry_constraints \
            else np.zeros(0, FACTOR_DTYPE)
        self.odom_only.append(self.prev_odom.copy())
        self.odom_at_last_align = self.prev_odom.copy()
        self._add_node(n, extra)
        return True

    def _add_node(self, n, extra, aligned=True):
        """updatePoseGraphObsConstraints (dpg_slam.cc:255-314) + optimizeGraph: the backend aligns the
        new node n with the preceding one and the preceding one with every earlier node within the
        distance rule (one batch), adds the factors and updates the graph."""
        extra = np.asarray(extra, FACTOR_DTYPE).reshape(-1)
        n_icp, X = self.be.add_node(self.clouds[n], self.node_pass, self.poses[n], extra,
                                    self.icp_params, self._reopt_params(), aligned and self.non_successive)
        self.n_factors += len(extra) + n_icp
        self.current_pass.append(n)
        self.poses = np.asarray(X, f32).reshape(-1, 3)

    def _reopt_params(self):
        rp = _abi.default_reopt_params()
        rp.max_node_dist_within_pass = float(self.within)
        rp.max_node_dist_across_passes = float(self.across)
        return rp

    def _dpg_store(self):
        """The node store over every node so far: created once, then the new nodes' scans are
        appended (dpg_dpg_append keeps the labels, sectors and activity of the others)."""
        V = len(self.poses)
        if self._store_V != V:
            rs = self.ranges[self._store_V:]
            offs = np.zeros(len(rs) + 1, np.int64)
            offs[1:] = np.cumsum([len(r) for r in rs])
            rng = np.ascontiguousarray(np.concatenate(rs), f32)
            geom = np.asarray(self.geom[self._store_V:], f32)
            if self._store is None:
                self._store = self.be.store(rng, geom, offs, self.change_params)
            else:
                self._store.append(rng, geom, offs)
            self._store_V = V
        return self._store
