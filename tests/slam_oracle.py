"""The CPU restatement behind DpgSLAM (dpgslam/slam.py) for the tests: the same backend methods as
slam.GpuBackend, computed by the oracle (oracle/, test infrastructure).  Per node it restates
dpg_add_node (dpg_api.hip; updatePoseGraphObsConstraints, dpg_slam.cc:255-314): the successive
pair and the loop-closure candidates (i, prev), i < V - 2, by the float distance rule, aligned one
by one by the oracle's ICP, the factors in the same order, then OracleIncGraph.update."""
import numpy as np

from dpgslam import _abi
from dpgslam.slam import _icp_factor
from oracle import oracle as O

f32 = np.float32


class OracleSlamBackend:
    def __init__(self, inc_mode="isam2"):
        self.g = O.OracleIncGraph(mode=inc_mode)
        self.clouds = []   # every node's base_link cloud, node order

    def add_node(self, cloud, passes, init_pose, extra, icp_params, reopt_params, non_successive):
        V = self.g.V
        self.clouds.append(np.asarray(cloud, f32))
        pf = np.concatenate([self.g.poses().astype(f32).reshape(-1, 3), np.asarray(init_pose, f32).reshape(1, 3)])
        edges = [(V - 1, V)] if V >= 1 else []
        if non_successive and V > 1:
            pv = V - 1
            for i in range(V - 2):
                dx, dy = f32(pf[i, 0] - pf[pv, 0]), f32(pf[i, 1] - pf[pv, 1])
                dist = np.sqrt(f32(f32(dx * dx) + f32(dy * dy)))
                thr = f32(reopt_params.max_node_dist_within_pass) if passes[i] == passes[pv] else \
                    f32(reopt_params.max_node_dist_across_passes)
                if dist <= thr:
                    edges.append((i, pv))
        F = [np.asarray(extra, _abi.FACTOR_DTYPE).reshape(-1)]
        n_icp = 0
        self.last_edges, self.last_results = edges, []
        for k, (a, b) in enumerate(edges):
            res, _, _ = O.run_icp(self.clouds[b], self.clouds[a], pf[b], pf[a], icp_params, O.NN_GRID)
            self.last_results.append(bytes(res))
            ok = bool(res.converged) and res.status == _abi.DPG_ICP_OK
            if k == 0 or ok:
                F.append(_icp_factor(res, a, b, icp_params))
                n_icp += 1
        self.g.update(np.asarray(init_pose, f32).astype(np.float64).reshape(1, 3), np.concatenate(F))
        return n_icp, self.g.poses()

    def icp_batch(self, clouds, edges, est, p):
        pts, offsets = clouds()
        return O.icp_batch(pts, offsets, edges, est, p, O.NN_GRID)[0]

    def candidates(self, est, passes, within, across):
        return O.loop_closure_candidates(est, passes, within, across)

    def rebuild_graph(self, est, F):
        self.g.reset()
        self.g.update(np.asarray(est, np.float64), F)
        return self.g.poses()

    def store(self, ranges, geom, offsets, params):
        return O.OracleDpgStore(ranges, geom, offsets=offsets, params=params)

    def get_map(self, clouds, est, fraction, ratio):
        pts, offsets = clouds()
        return O.get_map(pts, offsets, est, fraction)
