"""DPG change detection (DpgSLAM::executeDPG, dpg_slam.cc:865-886).

CPU tests pin the oracle restatement (oracle/dpg_change_oracle.cpp) with hand-built known answers
(no reference test or fixture covers this path, and the reference cannot be built here, so parity
against the reference itself is UNPINNED -- DESIGN.md §4).  GPU tests check the HIP path
(dpg-slam_amd/csrc/dpg_change.hip, through the C ABI) against the oracle bit for bit: every
counter, every point label, every sector bit and node flag after every call, and the four map lists.
"""
import math

import numpy as np
import pytest

from dpgslam import _abi, synth
from oracle import oracle as O

L_STATIC, L_ADDED, L_REMOVED, L_NYL, L_MAX = 0, 1, 2, 3, 4
NB = 360
AMIN, AMAX = -math.pi, math.pi


def _ring_scenario(extra_sector_range=None, near_sector_range=None, rmax=8.0):
    """Node 0 (pass 0) and node 1 (pass 1), same pose, in a round room of radius 5.  In pass 1 the
    beams of sector 0 (the first 72) either see beyond the old wall (`extra_sector_range`: the wall
    there was removed) or hit something new in front of it (`near_sector_range`)."""
    r = np.full((2, NB), 5.0, np.float32)
    if extra_sector_range is not None:
        r[1, :72] = extra_sector_range
    if near_sector_range is not None:
        r[1, :72] = near_sector_range
    geom = np.tile(np.array([AMIN, AMAX, rmax], np.float32), (2, 1))
    est = np.zeros((2, 3), np.float32)
    return r, geom, est


def _run(store_cls, r, geom, est, **kw):
    s = store_cls(r, geom, **kw) if store_cls is O.OracleDpgStore else store_cls(**kw)
    st = s.execute_dpg(2, 1, est)
    return s, st


def test_oracle_removed_wall_known_answer():
    r, geom, est = _ring_scenario(extra_sector_range=7.0)
    s = O.OracleDpgStore(r, geom)
    st = s.execute_dpg(2, 1, est)
    lab, sec, act = s.fetch()
    assert st.n_chain == 1 and st.n_candidates == 1 and st.n_submap_nodes == 1
    assert st.n_committed == 1 and st.n_added == 0
    removed = np.nonzero(lab[:NB] == L_REMOVED)[0]
    # the old wall points behind the new free rays, all in (or at the edge of) sector 0
    assert len(removed) == st.n_removed and 60 <= len(removed) <= 76
    assert removed.max() <= 73 and (removed < 72).sum() >= 60
    assert (lab[NB:] == L_NYL).all()                       # the current node keeps its labels
    assert not (sec[0] & 1)                                # sector 0 of node 0 went inactive
    assert act[0] == 1 and act[1] == 1                     # 4 of 5 sectors active >= 50 %
    assert st.n_sectors_deactivated == 1 and st.n_nodes_deactivated == 0


def test_oracle_new_object_known_answer():
    r, geom, est = _ring_scenario(near_sector_range=3.0)
    s = O.OracleDpgStore(r, geom)
    st = s.execute_dpg(2, 1, est)
    lab, sec, act = s.fetch()
    added = np.nonzero(lab[NB:] == L_ADDED)[0]
    assert st.n_committed == 1 and st.n_removed == 0
    assert len(added) == st.n_added and 60 <= len(added) <= 72 and added.max() < 72
    assert (lab[:NB] == L_NYL).all() and sec[0] == 0b11111 and sec[1] == 0b11111


def test_oracle_no_change_and_threshold():
    r, geom, est = _ring_scenario()
    s = O.OracleDpgStore(r, geom)
    st = s.execute_dpg(2, 1, est)
    assert st.n_added == 0 and st.n_removed == 0 and st.n_committed == 0
    assert st.n_uncovered == 0                             # the past node covers the whole chain grid
    # a change spanning 1/5 of the circle touches 8-9 of the 36 bins: committed at 0.2, not at 0.3
    r, geom, est = _ring_scenario(near_sector_range=3.0)
    p = _abi.default_change_params()
    p.delta_change_threshold = 0.3
    s = O.OracleDpgStore(r, geom, params=p)
    st = s.execute_dpg(2, 1, est)
    assert st.n_committed == 0 and st.n_added == 0


def test_oracle_greedy_submap_and_inactive_nodes():
    """Two identical past nodes: the second covers nothing new and stays out of the submap; an
    inactive past node is no candidate; coverage threshold 0 stops after the first candidate."""
    r = np.full((3, NB), 5.0, np.float32)
    geom = np.tile(np.array([AMIN, AMAX, 8.0], np.float32), (3, 1))
    est = np.zeros((3, 3), np.float32)
    s = O.OracleDpgStore(r, geom)
    st = s.execute_dpg(3, 1, est)
    assert st.n_candidates == 2 and st.n_submap_nodes == 1
    s.load(node_active=np.array([0, 1, 1], np.uint8))
    st = s.execute_dpg(3, 1, est)
    assert st.n_candidates == 1 and st.n_submap_nodes == 1
    p = _abi.default_change_params()
    p.current_pose_graph_coverage_threshold = 0.0
    s = O.OracleDpgStore(np.full((3, NB), 5.0, np.float32), geom, params=p)
    s.load(node_active=np.array([1, 1, 1], np.uint8))
    st = s.execute_dpg(3, 1, est)
    assert st.n_candidates == 2 and st.n_submap_nodes == 1


def test_oracle_map_lists():
    r, geom, est = _ring_scenario(extra_sector_range=7.0)
    s = O.OracleDpgStore(r, geom)
    s.execute_dpg(2, 1, est)
    lab, sec, act = s.fetch()
    m = s.active_dynamic_points(2, est)
    assert len(m["dynamic_removed"]) == int((lab == L_REMOVED).sum())
    assert len(m["active_static"]) == 0                      # nothing is ever labelled STATIC
    assert len(m["dynamic_added"]) == 0


def _dynamic(small=True):
    if small:
        return synth.make_dynamic(n_passes=3, nodes_per_pass=20, n_beams=NB, world_size=20.0, range_max=8.0,
                                  n_boxes=10)
    return synth.make_dynamic(n_passes=2, nodes_per_pass=40, n_beams=1000, seed=7, world_size=24.0,
                              range_max=12.0, n_boxes=12)


def test_oracle_dynamic_sequence_invariants():
    w = _dynamic()
    s = O.OracleDpgStore(w.ranges, w.geom)
    tot_rem = tot_add = 0
    for v in range(20, 60):
        p = w.pass_of[v]
        st = s.execute_dpg(v + 1, v - w.pass_start[p] + 1, w.est[:v + 1])
        assert 0 <= st.n_uncovered <= st.n_chain_cells
        assert st.n_submap_nodes <= st.n_candidates
        tot_rem += st.n_removed
        tot_add += st.n_added
    lab, sec, act = s.fetch()
    assert tot_add > 0 and tot_rem > 0
    assert 0 < int((lab == L_ADDED).sum()) <= tot_add   # chain nodes are re-tested while in the chain
    assert int((lab == L_REMOVED).sum()) <= tot_rem
    assert ((lab == L_MAX) == (w.ranges.reshape(-1) >= w.geom[0, 2])).all()


# ----------------------------------------------------------------------------------- GPU parity
def _gpu_store(r, geom, params=None):
    from dpgslam import api
    ctx = api.Context(0)
    return ctx, api.DpgStore(ctx, r, geom, params=params)


def _same_state(a, b):
    la, sa, aa = a.fetch()
    lb, sb, ab = b.fetch()
    assert np.array_equal(la, lb), f"labels differ at {np.nonzero(la != lb)[0][:10]}"
    assert np.array_equal(sa, sb), f"sectors differ at {np.nonzero(sa != sb)[0][:10]}"
    assert np.array_equal(aa, ab), f"node activity differs at {np.nonzero(aa != ab)[0][:10]}"


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["removed", "added", "none"])
def test_gpu_ring_known_answers(case):
    kw = {"removed": dict(extra_sector_range=7.0), "added": dict(near_sector_range=3.0), "none": {}}[case]
    r, geom, est = _ring_scenario(**kw)
    o = O.OracleDpgStore(r, geom)
    ctx, g = _gpu_store(r, geom)
    so = o.execute_dpg(2, 1, est)
    sg = g.execute_dpg(2, 1, est)
    assert sg.counters() == so.counters()
    _same_state(g, o)
    mo, mg = o.active_dynamic_points(2, est), g.active_dynamic_points(2, est)
    for k in mo:
        assert np.array_equal(mo[k], mg[k]), k


@pytest.mark.gpu
@pytest.mark.parametrize("small", [True, False])
def test_gpu_dynamic_sequence_parity(small):
    """Every executeDPG of the later passes, in order, on both paths: identical counters and state
    after each call, identical map lists at the end."""
    w = _dynamic(small)
    o = O.OracleDpgStore(w.ranges, w.geom)
    ctx, g = _gpu_store(w.ranges, w.geom)
    n0 = int(w.pass_start[1])
    calls = range(n0, w.V) if small else range(n0, w.V, 3)
    for v in calls:
        p = w.pass_of[v]
        cur = int(v - w.pass_start[p] + 1)
        so = o.execute_dpg(v + 1, cur, w.est[:v + 1])
        sg = g.execute_dpg(v + 1, cur, w.est[:v + 1])
        assert sg.counters() == so.counters(), (v, sg.counters(), so.counters())
        _same_state(g, o)
    mo, mg = o.active_dynamic_points(w.V, w.est), g.active_dynamic_points(w.V, w.est)
    for k in mo:
        assert np.array_equal(mo[k], mg[k]), k


@pytest.mark.gpu
def test_gpu_params_edges():
    """Chain longer than the pass, coverage threshold 0 (stop after one candidate), loaded state."""
    w = _dynamic()
    p = _abi.default_change_params()
    p.current_pose_graph_coverage_threshold = 0.0
    p.current_pose_chain_len = 8
    o = O.OracleDpgStore(w.ranges, w.geom, params=p)
    ctx, g = _gpu_store(w.ranges, w.geom, params=p)
    rng = np.random.default_rng(3)
    sec = rng.integers(0, 32, w.V).astype(np.uint8)
    act = (rng.random(w.V) < 0.8).astype(np.uint8)
    o.load(sector_active=sec, node_active=act)
    g.load(sector_active=sec, node_active=act)
    for v in (22, 27, 45, 59):
        pp = w.pass_of[v]
        cur = int(v - w.pass_start[pp] + 1)
        assert g.execute_dpg(v + 1, cur, w.est[:v + 1]).counters() == o.execute_dpg(v + 1, cur, w.est[:v + 1]).counters()
        _same_state(g, o)


def test_atan2f_restatement_matches_libm(tmp_path):
    """dpg_atan2f (the GPU's bearing function) == the host C library's atan2f on 40 M arguments and
    the special cases; run on the host (hipcc compiles the __host__ __device__ code for the CPU)."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "atan2f_check")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-ffp-contract=off", "-o", exe,
                    os.path.join(root, "tools", "atan2f_check.hip")], check=True, capture_output=True)
    out = subprocess.run([exe], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    assert "mismatches: 0 of" in out.stdout


@pytest.mark.gpu
def test_gpu_pose_updates_between_calls():
    """Estimates change between calls (as after a re-optimisation): the cached node frames and the
    kept chain planes must follow -- small perturbations every third call, one large shift that
    leaves the kept window, identical results to the oracle after every call."""
    w = _dynamic()
    o = O.OracleDpgStore(w.ranges, w.geom)
    ctx, g = _gpu_store(w.ranges, w.geom)
    rng = np.random.default_rng(11)
    est = w.est.copy()
    for n, v in enumerate(range(20, 60)):
        if n % 3 == 2:
            est[:v + 1, :2] += rng.normal(0, 0.02, (v + 1, 2)).astype(np.float32)
            est[:v + 1, 2] += rng.normal(0, 0.005, v + 1).astype(np.float32)
        if n == 25:
            est[:v + 1, 0] += np.float32(9.0)          # beyond the window margin: rebuild
        p = w.pass_of[v]
        cur = int(v - w.pass_start[p] + 1)
        so = o.execute_dpg(v + 1, cur, est[:v + 1])
        sg = g.execute_dpg(v + 1, cur, est[:v + 1])
        assert sg.counters() == so.counters(), (v, sg.counters(), so.counters())
        _same_state(g, o)
        if n % 3 == 2 or n == 25:   # the map lists after a pose change (inactive nodes' frames too)
            _same_map_lists(g, o, v + 1, est[:v + 1])
    # a node that went inactive while its pose changed, reactivated by dpg_dpg_load: its frame must
    # follow the pose it has now
    lab, sec, act = g.fetch()
    dead = np.nonzero(act[:60] == 0)[0][:3]
    if len(dead) < 3:   # make three nodes inactive if the sequence left fewer
        dead = np.array([5, 6, 7])
        act = act.copy()
        act[dead] = 0
        g.load(lab, sec, act)
        o.load(lab, sec, act)
    est[dead, :2] += np.float32(0.5)   # poses change while the nodes are inactive
    _same_map_lists(g, o, 60, est[:60])   # their removed / added points move with them
    act2, sec2 = act.copy(), sec.copy()
    act2[dead] = 1
    sec2[dead] = 0x1f
    g.load(lab, sec2, act2)
    o.load(lab, sec2, act2)
    _same_map_lists(g, o, 60, est[:60])


def _same_map_lists(g, o, n, est):
    a, b = g.active_dynamic_points(n, est), o.active_dynamic_points(n, est)
    for k in a:
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k


def _append_sequence(store_factory, w):
    """Create the store over the first pass, then append one node before each call (as the driver
    does while nodes are added)."""
    n0 = int(w.pass_start[1])
    s = store_factory(w.ranges[:n0], w.geom[:n0])
    out = []
    for v in range(n0, 60):
        s.append(w.ranges[v:v + 1], w.geom[v:v + 1])
        p = w.pass_of[v]
        st = s.execute_dpg(v + 1, int(v - w.pass_start[p] + 1), w.est[:v + 1])
        out.append((st.counters(), tuple(x.tobytes() for x in s.fetch())))
    return out


def test_oracle_append_equals_full_store():
    w = _dynamic()
    full = O.OracleDpgStore(w.ranges, w.geom)
    ref = []
    for v in range(int(w.pass_start[1]), 60):
        p = w.pass_of[v]
        st = full.execute_dpg(v + 1, int(v - w.pass_start[p] + 1), w.est[:v + 1])
        lab, sec, act = full.fetch()
        ref.append((st.counters(), (lab[:w.ranges[:v + 1].size].tobytes(), sec[:v + 1].tobytes(), act[:v + 1].tobytes())))
    got = _append_sequence(lambda r, g: O.OracleDpgStore(r, g), w)
    assert got == ref


@pytest.mark.gpu
def test_gpu_append_matches_oracle():
    from dpgslam import api
    w = _dynamic()
    ctx = api.Context(0)
    got = _append_sequence(lambda r, g: api.DpgStore(ctx, r, g), w)
    ref = _append_sequence(lambda r, g: O.OracleDpgStore(r, g), w)
    assert got == ref


# ------------------------------------------- reference placement of the pose chain (chain poses)
def _creation_poses(w, seed=3):
    """Stand-in for the reference's current_pass_nodes_ copies (dpg_slam.cc:195,307,598): the pose
    each node had when it was created (odometry-propagated), which optimizeGraph never refreshes --
    here the estimate plus a seeded drift that grows along the pass."""
    rng = np.random.default_rng(seed)
    c = w.est.astype(np.float64).copy()
    for p in range(len(w.pass_start) - 1):
        a, b = int(w.pass_start[p]), int(w.pass_start[p + 1])
        step = rng.normal(0.0, [0.01, 0.01, 0.002], size=(b - a, 3))
        c[a:b] += np.cumsum(step, axis=0)
    return c.astype(np.float32)


def _chain_of(w, creation, v, cur, chain_len=5):
    n = min(cur, chain_len)
    return creation[v + 1 - n:v + 1]


def test_oracle_chain_poses_at_estimates_equal_plain():
    w = _dynamic()
    a = O.OracleDpgStore(w.ranges, w.geom)
    b = O.OracleDpgStore(w.ranges, w.geom)
    for v in range(20, 60):
        p = w.pass_of[v]
        cur = int(v - w.pass_start[p] + 1)
        sa = a.execute_dpg(v + 1, cur, w.est[:v + 1])
        sb = b.execute_dpg(v + 1, cur, w.est[:v + 1], chain_poses=_chain_of(w, w.est, v, cur))
        assert sa.counters() == sb.counters(), v
    _same_state(a, b)


def test_oracle_chain_poses_drifted():
    """Chain grids at drifted creation poses against a submap at the estimates: the misalignment
    itself reads as change (DESIGN.md section 3, Q8 fix 8) -- more points labelled than with the
    chain at the estimates; the invariants hold either way."""
    w = _dynamic()
    cr = _creation_poses(w)
    a = O.OracleDpgStore(w.ranges, w.geom)
    b = O.OracleDpgStore(w.ranges, w.geom)
    ra = rb = 0
    for v in range(20, 60):
        p = w.pass_of[v]
        cur = int(v - w.pass_start[p] + 1)
        sa = a.execute_dpg(v + 1, cur, w.est[:v + 1])
        sb = b.execute_dpg(v + 1, cur, w.est[:v + 1], chain_poses=_chain_of(w, cr, v, cur))
        assert 0 <= sb.n_uncovered <= sb.n_chain_cells and sb.n_submap_nodes <= sb.n_candidates
        ra += sa.n_removed + sa.n_added
        rb += sb.n_removed + sb.n_added
    assert rb > ra


@pytest.mark.gpu
def test_gpu_chain_poses_parity():
    """dpg_execute_dpg_chain against the oracle bit for bit with drifted chain poses (every counter
    and the state after every call, the map lists at the end); with the chain at the estimates it
    equals dpg_execute_dpg."""
    w = _dynamic()
    cr = _creation_poses(w)
    o = O.OracleDpgStore(w.ranges, w.geom)
    ctx, g = _gpu_store(w.ranges, w.geom)
    g2 = __import__("dpgslam.api", fromlist=["api"]).DpgStore(ctx, w.ranges, w.geom)
    g3 = __import__("dpgslam.api", fromlist=["api"]).DpgStore(ctx, w.ranges, w.geom)
    for v in range(int(w.pass_start[1]), w.V):
        p = w.pass_of[v]
        cur = int(v - w.pass_start[p] + 1)
        ch = _chain_of(w, cr, v, cur)
        so = o.execute_dpg(v + 1, cur, w.est[:v + 1], chain_poses=ch)
        sg = g.execute_dpg(v + 1, cur, w.est[:v + 1], chain_poses=ch)
        assert sg.counters() == so.counters(), (v, sg.counters(), so.counters())
        _same_state(g, o)
        s2 = g2.execute_dpg(v + 1, cur, w.est[:v + 1])
        s3 = g3.execute_dpg(v + 1, cur, w.est[:v + 1], chain_poses=_chain_of(w, w.est, v, cur))
        assert s2.counters() == s3.counters(), v
    _same_state(g2, g3)
    mo, mg = o.active_dynamic_points(w.V, w.est), g.active_dynamic_points(w.V, w.est)
    for k in mo:
        assert np.array_equal(mo[k], mg[k]), k
