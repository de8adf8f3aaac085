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
    from slam_oracle import OracleSlamBackend
    w = synth.make_patrol(n_passes=2, steps=40)
    assert w.ranges.shape[1] == 5000
    so, sg = DpgSLAM(backend=OracleSlamBackend()), DpgSLAM(backend="gpu")
    to, tg, swo, swg = [], [], [], []
    _drive(so, w, to, swo)
    _drive(sg, w, tg, swg)
    assert to == tg                                    # same nodes and factors after every reading
    assert len(swo) == 1 and swo[0].shape == swg[0].shape
    assert np.abs(swo[0] - swg[0]).max() < 1e-5        # the sweep's poses
    assert np.abs(so.poses - sg.poses).max() < 1e-5
    lo, so_, ao = so._store.fetch()
    lg, sg_, ag = sg._store.fetch()
    assert np.array_equal(ao, ag) and (lo != lg).mean() < 1e-3
