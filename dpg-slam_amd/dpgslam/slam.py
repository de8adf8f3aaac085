"""DpgSLAM -- the public API of dpg_slam::DpgSLAM (src/dpg_slam/dpg_slam.h:283-335) as a host-side
driver over the MI355X C ABI: the per-node pipeline the ROS glue runs (ObserveOdometry,
ObserveLaser -> updatePoseGraph -> runIcp / optimizeGraph -> executeDPG, incrementPassNumber ->
reoptimize, GetPose, GetMap, getActiveAndDynamicMapPoints).

The bookkeeping (odometry thresholds, node creation, which scans are aligned, which factors are
added) follows dpg_slam.cc line by line in float32 where the reference is float; every numeric
step runs through a backend: "gpu" (the HIP kernels, dpgslam.api) or "oracle" (the CPU
restatement, test infrastructure), so tests can run the same driver on both and compare.
optimizeGraph runs batch Gauss-Newton to convergence over the accumulated graph instead of ISAM2's
single incremental update.
"""
from __future__ import annotations

import ctypes as C
import math

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


class _GpuBackend:
    def __init__(self, ctx: api.Context):
        self.ctx = ctx

    def run_icp(self, pose_1, cloud_1, pose_2, cloud_2, p):
        ok, z, cov, res, _ = self.ctx.run_icp(api.Node(pose_1, cloud_1), api.Node(pose_2, cloud_2), p)
        return bool(ok), res

    def icp_batch(self, pts, offsets, edges, est, p):
        self.ctx.upload_scans(pts, offsets, p.downsample_icp_points_ratio)
        res, _ = self.ctx.icp_batch(edges, est, p, compute_cov=False)
        return res

    def candidates(self, est, passes, within, across):
        return self.ctx.loop_closure_candidates(est, passes, within, across)

    def optimize(self, X0, F, gp):
        return self.ctx.optimize_graph(X0, F, gp)[0]

    def store(self, ranges, geom, offsets, params):
        return api.DpgStore(self.ctx, ranges, geom, offsets=offsets, params=params)

    def get_map(self, pts, offsets, est, fraction, ratio):
        self.ctx.upload_scans(pts, offsets, ratio)
        return self.ctx.get_map(est, fraction)


class _OracleBackend:
    def __init__(self):
        from oracle import oracle as O   # test infrastructure: the CPU restatement
        self.O = O

    def run_icp(self, pose_1, cloud_1, pose_2, cloud_2, p):
        res, _, _ = self.O.run_icp(cloud_2, cloud_1, pose_2, pose_1, p, self.O.NN_GRID)
        return bool(res.converged) and res.status == _abi.DPG_ICP_OK, res

    def icp_batch(self, pts, offsets, edges, est, p):
        return self.O.icp_batch(pts, offsets, edges, est, p, self.O.NN_GRID)[0]

    def candidates(self, est, passes, within, across):
        return self.O.loop_closure_candidates(est, passes, within, across)

    def optimize(self, X0, F, gp):
        return self.O.optimize_graph(X0, F, gp)[0]

    def store(self, ranges, geom, offsets, params):
        return self.O.OracleDpgStore(ranges, geom, offsets=offsets, params=params)

    def get_map(self, pts, offsets, est, fraction, ratio):
        return self.O.get_map(pts, offsets, est, fraction)


class DpgSLAM:
    """dpg_slam::DpgSLAM.  Parameters default to parameters.h (PoseGraphParameters, DpgParameters,
    VisualizationParams.display_points_fraction_)."""

    def __init__(self, backend="gpu", ctx: api.Context | None = None, icp_params=None, gn_params=None,
                 change_params=None, min_dist_between_nodes=1.0, min_angle_between_nodes=math.pi / 6.0,
                 non_successive_scan_constraints=True, odometry_constraints=True,
                 max_dist_within_pass=5.0, max_dist_across_passes=2.0, new_pass_std_dev=(0.2, 0.2, 0.15),
                 motion_model=(0.4, 0.4, 0.4, 0.4), display_points_fraction=10):
        if backend == "gpu":
            self.ctx = ctx or api.Context(0)
            self.be = _GpuBackend(self.ctx)
        elif backend == "oracle":
            self.be = _OracleBackend()
        else:
            raise ValueError(backend)
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
        self.poses: list[np.ndarray] = []               # dpg_nodes_ estimated positions (float32)
        self.node_pass: list[int] = []
        self.ranges: list[np.ndarray] = []
        self.geom: list[tuple] = []
        self.clouds: list[np.ndarray] = []
        self.odom_only: list[np.ndarray] = []
        self.current_pass: list[int] = []
        self.factors: list[np.ndarray] = []
        self._store = None
        self._store_V = 0

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
            self.executeDPG()

    def incrementPassNumber(self):
        """dpg_slam.cc:25-33."""
        self.pass_number += 1
        self.odom_initialized = False
        self.first_scan_for_pass = True
        self.current_pass = []
        self.reoptimize()

    def GetPose(self):
        """dpg_slam.cc:528-553: the last node's estimate plus the odometry not yet in the graph."""
        loc = self.poses[-1][:2] if self.poses else np.zeros(2, f32)
        ang = self.poses[-1][2] if self.poses else f32(0)
        un = self.prev_odom[:2] - self.odom_at_last_align[:2]
        dth = _angle_mod(self.prev_odom[2] - self.odom_at_last_align[2])   # AngleDiff
        disp = api.transform_point(np.array([un[0], un[1], 0], f32), np.array([0, 0, -self.odom_at_last_align[2]], f32))
        rot = api.transform_point(np.array([disp[0], disp[1], 0], f32), np.array([0, 0, ang], f32))
        return np.array([loc[0] + rot[0], loc[1] + rot[1]], f32), f32(ang + dth)

    def GetMap(self):
        """dpg_slam.cc:555-575."""
        if not self.poses:
            return np.zeros((0, 2), f32)
        pts, offs = self._clouds()
        return self.be.get_map(pts, offs, np.stack(self.poses), self.fraction,
                               self.icp_params.downsample_icp_points_ratio)

    def GetActiveAndDynamicMapPoints(self):
        """getActiveAndDynamicMapPoints (dpg_slam.cc:832-863) over the current node state."""
        return self._dpg_store().active_dynamic_points(len(self.poses), np.stack(self.poses))

    def executeDPG(self):
        """dpg_slam.cc:865-886 (dpg_execute_dpg on the node store)."""
        return self._dpg_store().execute_dpg(len(self.poses), len(self.current_pass), np.stack(self.poses))

    def reoptimize(self):
        """dpg_slam.cc:35-120: a fresh graph -- per node the pass prior or the odometry Between, the
        successive alignment (always a factor) and every loop-closure candidate (a factor when
        converged), all aligned in one batch from the current estimates -- then the solve."""
        V = len(self.poses)
        if V == 0:
            return
        est = np.stack(self.poses)
        passes = np.asarray(self.node_pass, np.int32)
        lc = self.be.candidates(est, passes, float(self.within), float(self.across))
        succ = np.stack([np.arange(V - 1), np.arange(1, V)], 1).astype(np.int32)
        edges = np.concatenate([succ, np.asarray(lc, np.int32).reshape(-1, 2)], 0)
        res = None
        if len(edges):
            pts, offs = self._clouds()
            res = self.be.icp_batch(pts, offs, edges, est, self.icp_params)
        F, cur = [], None
        for i in range(V):
            if i == 0 or passes[i] != cur:
                F.append(api.prior_factor(i, sigmas=self.prior_sigmas))
                cur = passes[i]
            elif self.odometry_constraints:
                F.append(self._odometry_factor(self.odom_only[i - 1], self.odom_only[i], i - 1, i))
        for k, (a, b) in enumerate(edges):
            ok = res["converged"][k] != 0 and res["status"][k] == _abi.DPG_ICP_OK
            if k < len(succ) or ok:
                F.append(_icp_factor(res[k:k + 1], int(a), int(b), self.icp_params))
        self.factors = F
        self._optimize()

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
        self.poses.append(np.asarray(pose, f32).copy())
        self.node_pass.append(self.pass_number)
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
            self.factors.append(api.prior_factor(n, sigmas=self.prior_sigmas))
            self.odom_only.append(self.prev_odom.copy())
            self.odom_at_last_align = self.prev_odom.copy()
            if self.pass_number == 0:
                self.current_pass.append(n)
                self._optimize()
                return False
            self._obs_constraints(n)
            return True
        if not self._should_process_laser():
            return False
        rel = api.inverse_transform_point(self.prev_odom, self.odom_at_last_align)   # displacement since the last node
        pose = api.transform_point(rel, self.poses[-1])                                # createRelativePositionedNode
        n = self._create_node(ranges, range_max, angle_min, angle_max, pose)
        if self.odometry_constraints:
            self.factors.append(self._odometry_factor(self.odom_at_last_align, self.prev_odom, n - 1, n))
        self.odom_only.append(self.prev_odom.copy())
        self.odom_at_last_align = self.prev_odom.copy()
        self._obs_constraints(n)
        return True

    def _obs_constraints(self, n):
        """updatePoseGraphObsConstraints (dpg_slam.cc:255-314); the new node n is already stored,
        so dpg_nodes_ of the reference is nodes [0, n)."""
        prev = n - 1
        ok, res = self.be.run_icp(self.poses[prev], self.clouds[prev], self.poses[n], self.clouds[n], self.icp_params)
        self.factors.append(_icp_factor(res, prev, n, self.icp_params))
        if self.non_successive and n > 1:
            pp = self.poses[prev]
            for i in range(max(0, n - 2)):
                d = self.poses[i][:2] - pp[:2]
                dist = f32(np.sqrt(f32(d[0] * d[0]) + f32(d[1] * d[1])))
                thr = self.within if self.node_pass[i] == self.node_pass[prev] else self.across
                if dist <= thr:
                    ok, res = self.be.run_icp(self.poses[i], self.clouds[i], pp, self.clouds[prev], self.icp_params)
                    if ok:
                        self.factors.append(_icp_factor(res, i, prev, self.icp_params))
        self.current_pass.append(n)
        self._optimize()

    def _optimize(self):
        """optimizeGraph (dpg_slam.cc:316-329): batch GN from the current estimates."""
        X0 = np.stack(self.poses).astype(np.float64)
        X = self.be.optimize(X0, np.concatenate(self.factors), self.gn_params)
        self.poses = [np.asarray(x, f32) for x in X]

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
