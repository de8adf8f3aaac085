"""Lockstep parity for DpgSLAM runs on the GPU (tests/test_slam.py, tests/test_config5.py): the GPU
backend runs the whole sequence, and at chosen steps the oracle TAKES OVER the GPU's state and
repeats that one step, which must then agree exactly -- so a tiny difference early in a long run
cannot hide behind the tolerance a free-running comparison needs (float poses: a 1e-13 solver
difference can flip an ulp and reroute later alignments).  Checked per sampled step:

* dpg_add_node (updatePoseGraphObsConstraints + optimizeGraph, dpg_slam.cc:255-329): the oracle
  restarts from the GPU graph's exported state (update count, factors, theta, estimate, max |delta|),
  derives the node's alignment pairs from the same estimates, aligns them (bit-exact results,
  edge for edge) and runs the ISAM2-semantics update (poses within POSE_TOL);
* executeDPG (dpg_slam.cc:865-886): the oracle node store loads the GPU store's labels / sectors /
  activity before the call, runs it, and must reproduce the counters and the whole state bit for bit;
* reoptimize (dpg_slam.cc:35-120): the loop-closure candidate set equal, a fixed sample of the
  sweep's alignments bit-exact, and the rebuilt graph's one update from the same factors within
  SWEEP_TOL."""
import numpy as np

from dpgslam import _abi
from dpgslam.slam import GpuBackend
from oracle import oracle as O
from slam_oracle import OracleSlamBackend

# a node's incremental update against the oracle's from the same state: every update solves the
# whole graph; the 80-node runs agree to 1e-13 - 1e-15, the 10 000-node patrol's updates after a
# pass-boundary sweep to ~1.4e-9 (the same conditioning effect as below, smaller steps)
POSE_TOL = 1e-8
# a sweep's update: ONE linear solve of the whole rebuilt graph (2 500 - 10 000 nodes, chains with a
# prior on each pass's first node only, condition numbers ~1e7-1e8): two correct fp64 Cholesky
# solves in different elimination orders differ by ~kappa * eps * |delta| (1.4e-8 measured at the
# 2 500-node sweep) -- still 70x inside north_star's 1e-6 pose tolerance
SWEEP_TOL = 1e-7


class _CheckedStore:
    """The GPU node store with the oracle's store beside it (kept structurally in step; its state is
    loaded from the GPU's before every sampled call)."""

    def __init__(self, owner, gpu_store, ranges, geom, offsets, params):
        self.o, self.g = owner, gpu_store
        self.orc = O.OracleDpgStore(ranges, geom, offsets=offsets, params=params)

    def append(self, ranges, geom, offsets=None):
        self.g.append(ranges, geom, offsets)
        self.orc.append(ranges, geom, offsets)

    def execute_dpg(self, n_nodes, current_pass_len, est, chain_poses=None):
        if not self.o.sample_dpg(n_nodes):
            return self.g.execute_dpg(n_nodes, current_pass_len, est, chain_poses)
        snap = self.g.fetch()
        sg = self.g.execute_dpg(n_nodes, current_pass_len, est, chain_poses)
        lab, sec, act = self.orc.fetch()
        lab[:len(snap[0])], sec[:len(snap[1])], act[:len(snap[2])] = snap
        self.orc.load(lab, sec, act)
        so = self.orc.execute_dpg(n_nodes, current_pass_len, est, chain_poses)
        assert sg.counters() == so.counters(), (n_nodes, sg.counters(), so.counters())
        for a, b in zip(self.g.fetch(), self.orc.fetch()):
            assert np.array_equal(a, b), f"executeDPG state differs after the call at {n_nodes} nodes"
        self.o.checked["dpg"] += 1
        return sg

    def __getattr__(self, name):
        return getattr(self.g, name)


class LockstepBackend(GpuBackend):
    """GpuBackend whose sampled steps are repeated by the oracle from the GPU's state.
    every: check the nodes whose id is a multiple of it (1: every node); dpg_every likewise for the
    executeDPG calls (by node count); sweep_sample: alignments of each sweep checked bit for bit."""

    def __init__(self, ctx, every=1, dpg_every=1, sweep_sample=64, inc_mode="isam2"):
        super().__init__(ctx, inc_mode)
        self.every, self.dpg_every, self.sweep_sample = int(every), int(dpg_every), int(sweep_sample)
        self.checked = {"nodes": 0, "icp": 0, "dpg": 0, "sweeps": 0, "sweep_icp": 0}
        self.max_pose_diff = 0.0
        self.node_diffs, self.sweep_diffs = [], []
        self.clouds_of = None   # set by the test: () -> every node's cloud, node order (DpgSLAM.clouds)
        self.inc_mode = inc_mode

    def sample_dpg(self, n_nodes):
        return (n_nodes - 1) % self.dpg_every == 0

    def add_node(self, cloud, passes, init_pose, extra, icp_params, reopt_params, non_successive):
        V = self.inc.V
        if V % self.every:
            return super().add_node(cloud, passes, init_pose, extra, icp_params, reopt_params, non_successive)
        st = self.inc.export_state()
        n_icp, X = super().add_node(cloud, passes, init_pose, extra, icp_params, reopt_params, non_successive)
        ob = OracleSlamBackend(self.inc_mode)
        ob.g.load_state(st)
        ob.clouds = list(self.clouds_of()[:V])
        n_o, Xo = ob.add_node(cloud, passes, init_pose, extra, icp_params, reopt_params, non_successive)
        if ob.last_edges:
            res, _ = self.ctx.icp_fetch(with_hessian=False)   # the node's batch stays staged
            assert len(res) == len(ob.last_edges), (V, len(res), len(ob.last_edges))
            for k, rb in enumerate(ob.last_results):
                assert res[k].tobytes() == rb, f"node {V}: alignment {k} {ob.last_edges[k]} differs from the oracle"
            self.checked["icp"] += len(res)
        assert n_icp == n_o, (V, n_icp, n_o)
        d = _pose_diff(X, Xo)
        self.max_pose_diff = max(self.max_pose_diff, d)
        self.node_diffs.append(d)
        assert d < POSE_TOL, f"node {V}: the update differs from the oracle's by {d:.3g}"
        self.checked["nodes"] += 1
        return n_icp, X

    def candidates(self, est, passes, within, across):
        lc = super().candidates(est, passes, within, across)
        ref = O.loop_closure_candidates(est, passes, within, across)
        assert np.array_equal(np.asarray(lc).reshape(-1, 2), np.asarray(ref).reshape(-1, 2)), "sweep candidates differ"
        return lc

    def icp_batch(self, clouds, edges, est, p):
        res = super().icp_batch(clouds, edges, est, p)
        k = min(self.sweep_sample, len(edges))
        if k:
            pick = np.unique(np.linspace(0, len(edges) - 1, k).round().astype(np.int64))
            pts, offsets = clouds()
            ref = O.icp_batch(pts, offsets, np.ascontiguousarray(edges[pick]), est, p, O.NN_GRID)[0]
            for q, e in enumerate(pick):
                assert res[e].tobytes() == ref[q].tobytes(), f"sweep alignment {e} {tuple(edges[e])} differs"
            self.checked["sweep_icp"] += len(pick)
        return res

    def rebuild_graph(self, est, F):
        X = super().rebuild_graph(est, F)
        g = O.OracleIncGraph(mode=self.inc_mode)
        g.update(np.asarray(est, np.float64), F)
        d = _pose_diff(X, g.poses())
        self.sweep_diffs.append(d)
        assert d < SWEEP_TOL, f"sweep update differs from the oracle's by {d:.3g}"
        self.checked["sweeps"] += 1
        return X

    def store(self, ranges, geom, offsets, params):
        return _CheckedStore(self, super().store(ranges, geom, offsets, params), ranges, geom, offsets, params)


def _pose_diff(A, B):
    A, B = np.asarray(A, np.float64).reshape(-1, 3), np.asarray(B, np.float64).reshape(-1, 3)
    d = A - B
    d[:, 2] = np.arctan2(np.sin(d[:, 2]), np.cos(d[:, 2]))
    return float(np.abs(d).max()) if len(d) else 0.0
