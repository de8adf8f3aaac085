"""Re-linearisation sweep (DpgSLAM::reoptimize, dpg_slam.cc:35-120): the GPU
loop-closure candidate search, and the whole sweep (candidates -> batched ICP -> factors -> batch
GN) against the oracle's restatement."""
import numpy as np
import pytest

from conftest import angle_wrap


def _passes(V, split):
    p = np.zeros(V, np.int32)
    p[split:] = 1
    return p


def test_candidate_rule_oracle_vs_kdtree(workload):
    """The oracle's O(V^2) candidate rule == an independent k-d tree formulation (float32 norm,
    <= threshold by pass), on config 2 with a pass boundary."""
    from scipy.spatial import cKDTree
    from oracle import oracle as O
    w = workload("config2")
    passes = _passes(w.V, 250)
    c = O.loop_closure_candidates(w.est, passes)
    xy = w.est[:, :2].astype(np.float64)
    pr = cKDTree(xy).query_pairs(5.0 * 1.001, output_type="ndarray")
    j, i = np.minimum(pr[:, 0], pr[:, 1]), np.maximum(pr[:, 0], pr[:, 1])
    keep = i - j >= 2
    j, i = j[keep], i[keep]
    d = w.est[j, :2] - w.est[i, :2]
    dist = np.sqrt(d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1])
    thr = np.where(passes[j] == passes[i], np.float32(5.0), np.float32(2.0))
    ok = dist <= thr
    ref = np.stack([j[ok], i[ok]], 1)
    ref = ref[np.lexsort((ref[:, 0], ref[:, 1]))]
    np.testing.assert_array_equal(c, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("split", [5000, 2500])
def test_gpu_candidates_match_oracle(ctx, workload, split):
    from oracle import oracle as O
    w = workload("config4")
    passes = _passes(w.V, split)
    g = ctx.loop_closure_candidates(w.est, passes)
    o = O.loop_closure_candidates(w.est, passes)
    assert len(o) > 0
    np.testing.assert_array_equal(g, o)


@pytest.mark.gpu
def test_gpu_candidates_edge_cases(ctx):
    from oracle import oracle as O
    for V in (1, 2, 3):
        est = np.zeros((V, 3), np.float32)
        assert len(ctx.loop_closure_candidates(est, np.zeros(V, np.int32))) == len(O.loop_closure_candidates(est, np.zeros(V, np.int32)))
    # exactly on the threshold (float): 5.0 is in, the next float above is out; across passes 2.0
    est = np.zeros((6, 3), np.float32)
    est[3, 0] = 5.0
    est[4, 0] = np.nextafter(np.float32(5.0), np.float32(6.0))
    est[5, 0] = 2.0
    passes = np.array([0, 0, 0, 0, 0, 1], np.int32)
    g = ctx.loop_closure_candidates(est, passes)
    np.testing.assert_array_equal(g, O.loop_closure_candidates(est, passes))
    assert [0, 3] in g.tolist() and [0, 4] not in g.tolist() and [0, 5] in g.tolist()


@pytest.mark.gpu
def test_reoptimize_matches_oracle(ctx, workload):
    """The whole sweep on 60 nodes of config 2 split into two passes: same candidate set and
    loop-closure decisions, poses within 1e-6 of the oracle's (GPU ICP is bit-exact, GN to
    max|delta| < 1e-10 on both sides)."""
    from oracle import oracle as O
    w = workload("config2")
    V = 60
    pts = w.pts[:w.offsets[V]]
    offs = w.offsets[:V + 1]
    passes = _passes(V, 30)
    ctx.upload_scans(pts, offs, 5)
    X, st = ctx.reoptimize(passes, w.est[:V], w.odom[:V])
    Xo, edges, res, so = O.reoptimize(pts, offs, passes, w.est[:V], w.odom[:V])
    assert st.n_icp_edges == len(edges) and st.n_candidates == len(edges) - (V - 1)
    conv = (res["converged"][V - 1:] != 0) & (res["status"][V - 1:] == 0)
    assert st.n_loop_closures == int(conv.sum()) and st.n_loop_closures > 0
    err = np.abs(np.concatenate([X[:, :2] - Xo[:, :2], angle_wrap(X[:, 2:] - Xo[:, 2:])], 1)).max()
    assert err < 1e-6, err
    assert st.gn.iterations < 100


@pytest.mark.gpu
def test_get_map_bit_exact(ctx, workload):
    """GetMap (dpg_slam.cc:555-575) on config 2's 500 full clouds (2.5 M points): every kept point
    bit-identical to the oracle's transformPoint, fraction 10 (parameters.h:22) and 7."""
    from oracle import oracle as O
    w = workload("config2")
    ctx.upload_scans(w.pts, w.offsets, 5)
    for frac in (10, 7):
        g = ctx.get_map(w.est, frac)
        o = O.get_map(w.pts, w.offsets, w.est, frac)
        assert g.shape == o.shape and g.tobytes() == o.tobytes()


@pytest.mark.gpu
def test_reoptimize_inc_rebuilds_the_live_graph(ctx, workload):
    """dpg_reoptimize_inc: the sweep on a live incremental graph rebuilds it from the sweep's
    factors (the reference's new ISAM2 + graph_, dpg_slam.cc:36-39,111-119).  In batch mode its
    single update runs GN to convergence, so the poses equal the oracle's sweep to 1e-6; the graph
    then keeps growing by dpg_add_node on top of the swept graph."""
    from dpgslam import api
    from oracle import oracle as O
    w = workload("config2")
    V = 60
    pts, offs = w.pts[:w.offsets[V]], w.offsets[:V + 1]
    passes = _passes(V, 30)
    ctx.upload_scans(pts, offs, 5)
    g = api.IncGraph(ctx, mode="batch")
    X, st = g.reoptimize(passes, w.est[:V], w.odom[:V])
    Xo, edges, res, so = O.reoptimize(pts, offs, passes, w.est[:V], w.odom[:V])
    assert g.V == V and st.n_icp_edges == len(edges) and st.n_loop_closures > 0
    err = np.abs(np.concatenate([X[:, :2] - Xo[:, :2], angle_wrap(X[:, 2:] - Xo[:, 2:])], 1)).max()
    assert err < 1e-6, err
    np.testing.assert_array_equal(g.poses(), X)
    p2 = np.append(passes, np.int32(1))
    s2 = g.add_node(w.cloud(V), p2, w.est[V])
    assert g.V == V + 1 and s2.n_icp_edges >= 1
    g.close()


@pytest.mark.gpu
def test_reoptimize_pass_boundary_patrol_at_size(ctx):
    """One pass-boundary sweep at size: the patrol workload of config 5 (5000-beam,
    270-degree, 30 m scans of a serpentine route; bench.py --workload dynamic), 2 x 1300 readings as
    nodes -- 2600 nodes over two passes, every node's cloud uploaded, the estimates = ground truth
    perturbed by odometry-scale noise.  Against the oracle's restatement (its ICP over 16 threads):
    the loop-closure candidate set and the sweep's own ICP results of every edge (fetched from the
    batch dpg_reoptimize ran) bit for bit, the poses < 1e-6."""
    from dpgslam import _abi, api, synth
    from oracle import oracle as O
    w = synth.make_patrol(n_passes=2, steps=1300)
    V = 2 * w.steps
    amin, amax, rmax = (float(x) for x in w.geom[0])
    pts, offs = api.scans_to_clouds(w.ranges, amin, amax, rmax)
    gtm = w.gt_map().reshape(-1, 3)
    rng = np.random.default_rng(11)
    est = (gtm + rng.normal(0.0, [0.05, 0.05, 0.01], gtm.shape)).astype(np.float32)
    passes = np.repeat(np.arange(2, dtype=np.int32), w.steps)
    odom = w.odom.reshape(-1, 3)
    p = _abi.default_icp_params()
    ctx.upload_scans(pts, offs, p.downsample_icp_points_ratio)
    cand_g = ctx.loop_closure_candidates(est, passes)
    cand_o = O.loop_closure_candidates(est, passes)
    np.testing.assert_array_equal(cand_g, cand_o)
    assert len(cand_o) > 2 * V   # within-pass neighbours along the route and the second pass's revisits
    X, st = ctx.reoptimize(passes, est, odom)
    Xo, edges, res_o, so = O.reoptimize(pts, offs, passes, est, odom, threads=16)
    assert st.n_icp_edges == len(edges) and st.n_candidates == len(cand_o)
    # the sweep's OWN alignments (its batch stays staged after dpg_reoptimize), not a re-run
    res_g, _ = ctx.icp_fetch(with_hessian=False)
    assert len(res_g) == len(edges)
    assert res_g.tobytes() == res_o.tobytes(), "the sweep's ICP results differ from the oracle's"
    conv = (res_o["converged"][V - 1:] != 0) & (res_o["status"][V - 1:] == 0)
    assert st.n_loop_closures == int(conv.sum())
    err = np.abs(np.concatenate([X[:, :2] - Xo[:, :2], angle_wrap(X[:, 2:] - Xo[:, 2:])], 1)).max()
    assert err < 1e-6, err
