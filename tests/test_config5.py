"""Config 5 (BASELINE configs[4]: "10k-node graph with DPG node removal + re-linearisation sweep")
at full scan geometry -- 5000-beam, 270-degree, 30 m scans -- against the oracle:

* a contiguous block of executeDPG calls (dpg_slam.cc:865-886) at the start of pass 1 over a
  300-node pass 0 of the non-collapsing workload (bench.py --workload dpg), whose first calls see
  70-105 submap candidates: counters after every call and the whole node state after the block
  bit for bit;
* DpgSLAM end to end on the patrol workload (bench.py --workload dynamic): two passes, per node
  dpg_add_node + executeDPG, the reoptimize sweep at the pass boundary (dpg_slam.cc:25-120) --
  GPU backend against the oracle backend: the same nodes and factors after every reading, the
  sweep poses and the final poses, and the DPG state (tolerances as tests/test_slam.py, which
  explains them)."""
import numpy as np
import pytest

from dpgslam import api, synth
from dpgslam.slam import DpgSLAM

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = api.Context(0)
    yield c
    c.close()


def test_config5_dpg_block_full_geometry(ctx):
    from oracle import oracle as O
    w = synth.make_dynamic(n_passes=2, nodes_per_pass=300, world_size=64.0, fov_deg=270.0, n_boxes=48,
                           range_noise=0.0)
    assert w.ranges.shape[1] == 5000 and float(w.geom[0, 2]) == 30.0
    g = api.DpgStore(ctx, w.ranges, w.geom)
    o = O.OracleDpgStore(w.ranges, w.geom)
    s0 = int(w.pass_start[1])
    cands = []
    for v in range(s0, s0 + 8):
        sg = g.execute_dpg(v + 1, v - s0 + 1, w.est[:v + 1])
        so = o.execute_dpg(v + 1, v - s0 + 1, w.est[:v + 1])
        assert sg.counters() == so.counters(), (v, sg.counters(), so.counters())
        cands.append(sg.n_candidates)
    assert max(cands) >= 50, cands
    for a, b in zip(g.fetch(), o.fetch()):
        assert np.array_equal(a, b)
    g.close()


def _drive(slam, w, trace, sweeps):
    amin, amax, rmax = (float(x) for x in w.geom[0])
    for p in range(w.n_passes):
        if p:
            slam.incrementPassNumber()
            sweeps.append(slam.poses.copy())
        for k in range(w.steps):
            o = w.odom[p, k]
            slam.ObserveOdometry(o[:2], o[2])
            slam.ObserveLaser(w.ranges[p * w.steps + k], 0.0, rmax, amin, amax)
            trace.append((len(slam.poses), slam.n_factors))


def test_config5_slam_sweep_full_geometry():
    """Two passes of the patrol at full scan geometry, GPU against the oracle in lockstep at every
    node, every executeDPG call and the pass-boundary sweep (tests/slam_lockstep.py); a free-running
    oracle run gives the same nodes and factors after every reading."""
    from slam_lockstep import LockstepBackend
    from slam_oracle import OracleSlamBackend
    w = synth.make_patrol(n_passes=2, steps=40)
    assert w.ranges.shape[1] == 5000
    so = DpgSLAM(backend=OracleSlamBackend())
    to, tg, swo, swg = [], [], [], []
    _drive(so, w, to, swo)
    with api.Context(0) as ctx:   # its own scan store
        be = LockstepBackend(ctx, every=1, dpg_every=1, sweep_sample=10 ** 6)
        sg = DpgSLAM(backend=be, ctx=ctx)
        be.clouds_of = lambda: sg.clouds
        _drive(sg, w, tg, swg)
    assert to == tg                                    # same nodes and factors after every reading
    V = len(sg.poses)
    n_later = int(np.sum(np.asarray(sg.node_pass) >= 1))
    assert be.checked["nodes"] == V and be.checked["sweeps"] == 1 and be.checked["dpg"] == n_later, be.checked
    print("lockstep", be.checked, "max pose diff", be.max_pose_diff)


@pytest.mark.slow
def test_config5_10k_lockstep():
    """BASELINE config 5 at its stated size: DpgSLAM over the 4 x 2500-reading patrol (10 000 nodes)
    on the GPU -- per node dpg_add_node, executeDPG from pass 1 on, the reoptimize sweep at every pass
    boundary and once more at 10 k nodes (dpg_slam.cc:25-120,255-329,865-886) -- with the oracle in
    lockstep on a fixed sample: every 250th node (its alignments bit-exact, its update within 1e-8 of
    the oracle's from the GPU's state, tests/slam_lockstep.py POSE_TOL), every 250th executeDPG call (counters and node state bit for
    bit), and each sweep (candidate set equal, 64 of its alignments bit-exact, its update within
    1e-7: one solve of the whole ill-conditioned graph, tests/slam_lockstep.py SWEEP_TOL)."""
    import time
    from slam_lockstep import LockstepBackend
    t0 = time.time()
    w = synth.make_patrol(n_passes=4, steps=2500)
    trace, sweeps = [], []
    with api.Context(0) as ctx:   # its own scan store
        be = LockstepBackend(ctx, every=250, dpg_every=250, sweep_sample=64)
        sg = DpgSLAM(backend=be, ctx=ctx)
        be.clouds_of = lambda: sg.clouds
        _drive(sg, w, trace, sweeps)
        sg.reoptimize()                                # the sweep at 10 k nodes
    V = len(sg.poses)
    assert V == 10000 and len(sweeps) == 3
    later = np.nonzero(np.asarray(sg.node_pass) >= 1)[0] + 1          # node counts at the executeDPG calls
    assert be.checked["nodes"] == 40 and be.checked["sweeps"] == 4, be.checked
    assert be.checked["dpg"] == int(np.sum((later - 1) % 250 == 0)) >= 25, be.checked
    assert be.checked["sweep_icp"] == 4 * 64 and be.checked["icp"] >= 40
    print(f"config5 10k lockstep in {time.time() - t0:.0f} s:", be.checked, "node update diffs max",
          max(be.node_diffs), "sweep diffs", be.sweep_diffs)
