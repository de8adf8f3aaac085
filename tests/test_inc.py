"""Incremental per-node solve (dpg_slam.cc:255-329 optimizeGraph -> isam_->update):
the incremental symbolic analysis (kept order, fill added along the elimination tree) against a
from-scratch elimination, the oracle's ISAM2/batch restatement against known answers, and the GPU
graph (dpg_inc) against the oracle node by node."""
import os
import subprocess

import numpy as np
import pytest

from dpgslam import _abi, synth
from oracle import oracle as O
from graphs import gtsam_test_graph, pose_diff

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def incsym_bin(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("incsym") / "incsym_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", out, os.path.join(ROOT, "tools", "incsym_check.cpp"),
                    os.path.join(ROOT, "dpg-slam_amd", "csrc", "dpg_chol_sym.cpp")], check=True)
    return out


@pytest.mark.parametrize("n0,steps,seed,split", [(200, 150, 1, ""), (500, 200, 7, ""), (64, 300, 3, ""),
                                                 (30, 120, 11, ""), (400, 120, 5, "split")])
def test_incremental_symbolic_matches_elimination(incsym_bin, n0, steps, seed, split):
    r = subprocess.run([incsym_bin, str(n0), str(steps), str(seed)] + ([split] if split else []), capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.parametrize("n0,steps,seed,split,lead", [(500, 120, 9, "-", 8), (300, 100, 4, "split", 16),
                                                      (260, 80, 2, "-", 40)])
def test_background_order_extended_matches_elimination(incsym_bin, n0, steps, seed, split, lead):
    """The background reorder's state (dpg_inc.hip): the order of a snapshot taken `lead` nodes
    earlier, extended by the nodes and edges since, keeps column patterns equal to a from-scratch
    elimination of the whole graph in that order, through later growth."""
    r = subprocess.run([incsym_bin, str(n0), str(steps), str(seed), split, str(lead)], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr


@pytest.mark.parametrize("n,seed", [(3000, 1), (6000, 2), (9000, 3)])
def test_threaded_nested_dissection_gives_the_serial_order(tmp_path, n, seed):
    """The orderings' threaded forms (a large part's halves on two threads, its separator starts on
    up to four, level structures reused) give the serial permutation and column patterns, for both
    candidate rules and the incremental reorder (dpg_chol_sym.cpp), on route-like graphs of 1-3
    components."""
    out = str(tmp_path / "nd_par_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-o", out, os.path.join(ROOT, "tools", "nd_par_check.cpp"),
                    os.path.join(ROOT, "dpg-slam_amd", "csrc", "dpg_chol_sym.cpp")], check=True)
    r = subprocess.run([out, str(n), str(seed)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr


def test_solver_plan_matches_straightforward_construction(tmp_path):
    """The GPU solver's host plan (dpg_chol.hip chol_plan: H-block -> front map by column buckets,
    child column ranges by binary search, critical-path front order) equals the straightforward
    construction (per-block binary search + per-front sort, linear scans, stable sort) after every
    update of a growing graph: tools/incsym_bench.cpp built with DPG_PLAN_VERIFY aborts on the first
    difference -- including the H-block buckets the incremental prepare builds ahead from the
    incremental state's order (dpg_chol_plan_blocks, every 50th update) and that order against the
    analysis's.  Host code only (hipcc compiles it; no device call runs)."""
    exe = str(tmp_path / "incsym_bench_v")
    csrc = os.path.join(ROOT, "dpg-slam_amd", "csrc")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17", "-ffp-contract=off",
                    "-DDPG_PLAN_VERIFY", "-o", exe, os.path.join(ROOT, "tools", "incsym_bench.cpp"),
                    os.path.join(csrc, "dpg_chol.hip"), os.path.join(csrc, "dpg_chol_sym.cpp")], check=True)
    rng = np.random.default_rng(5)
    V, buf = 700, [700]
    for v in range(V):
        e = [(v - 1, v)] if v else []
        for _ in range(rng.integers(0, 4) if v > 20 else 0):
            e.append((int(rng.integers(0, v - 10)), v))
        e = sorted(set(e))
        buf.append(len(e))
        buf.extend(x for p in e for x in p)
    path = str(tmp_path / "edges.bin")
    np.asarray(buf, np.int32).tofile(path)
    r = subprocess.run([exe, path, "50", "32", "1.5"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "V=700" in r.stdout, r.stdout + r.stderr


def _per_node(F):
    """Factors grouped by the update that adds them: the one whose largest key is the new node."""
    key = np.maximum(F["i"], np.where(F["kind"] == _abi.DPG_FACTOR_BETWEEN, F["j"], -1))
    return key


def test_oracle_incremental_batch_mode_reaches_gtsam_test_optimum():
    X0, F, X_opt = gtsam_test_graph()
    g = O.OracleIncGraph(mode="batch")
    key = _per_node(F)
    for v in range(len(X0)):
        g.update(X0[v:v + 1], F[key == v])
    assert np.abs(pose_diff(g.poses(), X_opt)).max() < 1e-9


def test_oracle_incremental_isam2_relinearization():
    """ISAM2 mode takes one step per update from lagging linearization points.  With threshold 0
    every 10th update relinearizes everything, and empty updates converge to the batch optimum;
    with the default 0.1 relinearization stops once every |delta| < 0.1 and the estimate stays the
    linearized solution theta (+) delta (GTSAM's behaviour), close to but not at the optimum."""
    X0, F, X_opt = gtsam_test_graph()
    key = _per_node(F)
    g0 = O.OracleIncGraph(mode="isam2", relinearize_threshold=0.0)
    g = O.OracleIncGraph(mode="isam2")
    for v in range(len(X0)):
        g0.update(X0[v:v + 1], F[key == v])
        g.update(X0[v:v + 1], F[key == v])
    snap = None
    for k in range(60):
        g0.update(np.zeros((0, 3)), F[:0])
        g.update(np.zeros((0, 3)), F[:0])
        if k == 30:
            snap = g.poses()
    assert np.abs(pose_diff(g0.poses(), X_opt)).max() < 1e-9
    assert g.maxd.max() < 0.1 and np.array_equal(g.poses(), snap)
    assert 1e-9 < np.abs(pose_diff(g.poses(), X_opt)).max() < 1e-3


def _sequence(name, n_nodes):
    """A per-node factor sequence from a synthetic workload: node v arrives with its odometry and
    successive ICP factors and the loop closures (j, v), j < v, measured by the oracle's ICP."""
    w = synth.generate(name)
    E = w.edges
    sel = E[:, 1] < n_nodes
    res, _ = O.icp_batch(w.pts, w.offsets, E[sel], w.est, None, O.NN_GRID, min(8, os.cpu_count() or 1))
    full = np.zeros(w.E, _abi.RESULT_DTYPE)
    full[sel] = res
    F = w.factors_with_icp(full)
    keep = np.concatenate([np.ones(len(w.base_factors), bool), sel])
    F = F[keep]
    F = F[_per_node(F) < n_nodes]
    return w.est[:n_nodes].astype(np.float64), F


@pytest.mark.gpu
@pytest.mark.parametrize("mode,dup", [("isam2", False), ("batch", False), ("isam2", True)])
def test_gpu_incremental_matches_oracle(ctx, mode, dup):
    from dpgslam import api
    X0, F = _sequence("config3", 600 if mode != "batch" else 300)
    key = _per_node(F)
    g = api.IncGraph(ctx, mode=mode, duplicate_factors=dup, reorder_every=64)
    o = O.OracleIncGraph(mode=mode, duplicate_factors=dup)
    worst = 0.0
    reorders = 0
    for v in range(len(X0)):
        st = g.update(X0[v:v + 1], F[key == v])
        o.update(X0[v:v + 1], F[key == v])
        reorders += st.reordered
        if v % 25 == 0 or v == len(X0) - 1:
            d = np.abs(pose_diff(g.poses(), o.poses())).max()
            worst = max(worst, d)
    assert worst < 1e-6, worst
    assert reorders < len(X0) / 8   # the order is extended, not recomputed
    g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("reorder_every", [32, 64])
def test_gpu_partial_refactor_is_bit_identical(ctx, reorder_every):
    """ISAM2's partial re-elimination (isam_->update, dpg_slam.cc:320): an update refactors only the
    Cholesky fronts its new nodes, factors and pairs touch and their ancestors, and keeps the rest.
    Every estimate, error and delta equals the full refactorization's bit for bit -- through
    loop closures, relinearizations (updates 10, 20, ...), reorders and updates without new nodes --
    and most updates keep most fronts."""
    from dpgslam import api
    X0, F = _sequence("config3", 400)
    key = _per_node(F)
    gp = api.IncGraph(ctx, reorder_every=reorder_every)
    gf = api.IncGraph(ctx, reorder_every=reorder_every, full_refactor=True)
    kept_updates = 0
    n_upd = 0
    for v in range(len(X0) + 12):
        x = X0[v:v + 1] if v < len(X0) else np.zeros((0, 3))
        f = F[key == v] if v < len(X0) else F[:0]
        sp = gp.update(x, f)
        sf = gf.update(x, f)
        n_upd += 1
        assert sf.fronts_kept == 0
        kept_updates += sp.fronts_kept > 0
        assert (sp.error, sp.last_delta_inf, sp.relinearized) == (sf.error, sf.last_delta_inf, sf.relinearized), v
        if v % 20 == 0 or v >= len(X0) - 2:
            assert np.array_equal(gp.poses(), gf.poses()), v
    assert np.array_equal(gp.export_state()["theta"], gf.export_state()["theta"])
    assert kept_updates > n_upd // 2, (kept_updates, n_upd)
    gp.close()
    gf.close()


@pytest.mark.gpu
def test_gpu_partial_refactor_through_failed_updates(ctx):
    """Failed updates (a node without factors: H singular) roll the graph back; the partial path
    forgets its tracked factorization and the next updates still equal the full refactorization's
    bit for bit, including updates that keep fronts again afterwards."""
    from dpgslam import api
    X0, F = _sequence("config3", 160)
    key = _per_node(F)
    gp = api.IncGraph(ctx, reorder_every=64)
    gf = api.IncGraph(ctx, reorder_every=64, full_refactor=True)
    kept_after = 0
    for v in range(len(X0)):
        if v in (41, 42, 97):
            for g in (gp, gf):
                with pytest.raises(_abi.DpgError):
                    g.update(X0[v:v + 1], F[:0])
        sp = gp.update(X0[v:v + 1], F[key == v])
        sf = gf.update(X0[v:v + 1], F[key == v])
        if v > 97:
            kept_after += sp.fronts_kept > 0
        assert (sp.error, sp.last_delta_inf) == (sf.error, sf.last_delta_inf), v
    assert np.array_equal(gp.poses(), gf.poses())
    assert kept_after > 20, kept_after
    gp.close()
    gf.close()


def test_oracle_isam2_first_relinearization_is_update_10():
    """ISAM2::update counts the update before relinarizationNeeded(update_count_) (GTSAM 4.0), so
    with relinearizeSkip 10 the linearization points first move on the 10th update, then the 20th
    -- never on updates 1-9 or 11-19 (threshold 0: every variable with a nonzero delta moves)."""
    X0, F, _ = gtsam_test_graph()
    key = _per_node(F)
    g = O.OracleIncGraph(mode="isam2", relinearize_threshold=0.0)
    moved = []
    for u in range(1, 26):
        before = g.theta.copy()
        if u <= len(X0):
            g.update(X0[u - 1:u], F[key == u - 1])
        else:
            g.update(np.zeros((0, 3)), F[:0])
        n0 = len(before)
        if n0 and not np.array_equal(g.theta[:n0], before):
            moved.append(u)
    assert moved == [10, 20], moved


@pytest.mark.gpu
def test_gpu_failed_update_rolls_back(ctx):
    """A numeric failure (a node with no factor: H singular) leaves the device graph as it was --
    node count, factors, pattern, estimate -- and the next updates proceed and still match the
    oracle (the failure used to leave the graph one node ahead of itself)."""
    from dpgslam import api
    X0, F = _sequence("config3", 120)
    key = _per_node(F)
    g = api.IncGraph(ctx, mode="isam2", reorder_every=16)
    o = O.OracleIncGraph(mode="isam2")
    for v in range(len(X0)):
        if v in (30, 77):   # the injected failure: the node arrives without its factors
            before = g.poses()
            with pytest.raises(_abi.DpgError):
                g.update(X0[v:v + 1], F[:0])
            assert g.V == v and np.array_equal(g.poses(), before)
        g.update(X0[v:v + 1], F[key == v])
        o.update(X0[v:v + 1], F[key == v])
    assert np.abs(pose_diff(g.poses(), o.poses())).max() < 1e-6
    g.close()


@pytest.mark.gpu
def test_gpu_add_node_failure_keeps_store_and_graph_in_step():
    """dpg_add_node_pairs with no factor for the new node fails in the update; the scan store drops
    the node again (store and graph keep the same count) and the next dpg_add_node succeeds."""
    from dpgslam import api
    w = synth.generate("config2")
    p = _abi.default_icp_params()
    ctx = api.Context(0)   # a fresh scan store
    g = api.IncGraph(ctx, mode="isam2")
    prior = np.zeros(1, _abi.FACTOR_DTYPE)
    prior["kind"], prior["i"], prior["info"] = _abi.DPG_FACTOR_PRIOR, 0, 1.0 / np.array([0.04, 0.04, 0.0225])
    g.add_node(w.cloud(0), np.zeros(1, np.int32), w.est[0], extra=prior, icp_params=p)
    g.add_node(w.cloud(1), np.zeros(2, np.int32), w.est[1], icp_params=p)
    with pytest.raises(_abi.DpgError):   # no successive alignment, no pairs, no factor: singular
        g.add_node_pairs(w.cloud(2), w.est[2], np.zeros((0, 2), np.int32), successive=False, icp_params=p)
    assert g.V == 2
    st = g.add_node(w.cloud(2), np.zeros(3, np.int32), w.est[2], icp_params=p)
    assert g.V == 3 and st.n_icp_edges >= 1
    g.close()
    ctx.close()


@pytest.mark.gpu
def test_gpu_fetch_capacity_checked_after_add_node():
    """dpg_icp_batch_fetch takes the capacity of the caller's buffers: after
    dpg_add_node_pairs stages a batch of several alignments inside C, a buffer one record short is
    refused with DPG_ERR_SIZE and left untouched (no heap damage), and the exact size succeeds.
    dpg_icp_batch_fetch_trace likewise refuses a short trace buffer."""
    import ctypes as C
    from dpgslam import api
    from dpgslam._abi import lib
    from dpgslam.api import results_array
    w = synth.generate("config2")
    p = _abi.default_icp_params()
    ctx = api.Context(0)
    g = api.IncGraph(ctx, mode="isam2")
    prior = np.zeros(1, _abi.FACTOR_DTYPE)
    prior["kind"], prior["i"], prior["info"] = _abi.DPG_FACTOR_PRIOR, 0, 1.0 / np.array([0.04, 0.04, 0.0225])
    g.add_node(w.cloud(0), np.zeros(1, np.int32), w.est[0], extra=prior, icp_params=p)
    g.add_node(w.cloud(1), np.zeros(2, np.int32), w.est[1], icp_params=p)
    g.add_node_pairs(w.cloud(2), w.est[2], np.array([[0, 2]], np.int32), successive=True, icp_params=p)
    n = int(lib().dpg_icp_batch_size(ctx.handle))
    assert n == 2, n
    short = results_array(n + 1)
    sentinel = short.tobytes()
    hess = np.full((n + 1, 9), -7.0)
    rc = lib().dpg_icp_batch_fetch(ctx.handle, short.ctypes.data_as(C.c_void_p),
                                   hess.ctypes.data_as(C.POINTER(C.c_double)), n - 1)
    assert rc == -4 and short.tobytes() == sentinel and (hess == -7.0).all()   # DPG_ERR_SIZE
    assert b"staged batch" in (lib().dpg_last_error() or b"")
    res, _ = ctx.icp_fetch(with_hessian=False)     # the exact size: the two alignments
    assert len(res) == n and all(int(r["iterations"]) > 0 for r in res)
    # a NULL-pointer fetch needs no capacity (it only feeds the cost memory)
    assert lib().dpg_icp_batch_fetch(ctx.handle, None, None, 0) == 0
    g.close()
    ctx.close()
    # the trace: one int32 short of E * trace_iters * max_src is refused
    ctx = api.Context(0)
    ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
    ctx.icp_prepare(w.edges[:3], w.est, p)
    ctx.icp_run(compute_cov=False, trace_iters=2)
    ms = C.c_int64(0)
    assert lib().dpg_icp_batch_fetch_trace(ctx.handle, None, 0, C.byref(ms)) == 0
    need = 3 * 2 * ms.value
    tr = np.full(need, -5, np.int32)
    rc = lib().dpg_icp_batch_fetch_trace(ctx.handle, tr.ctypes.data_as(C.POINTER(C.c_int32)), need - 1, C.byref(ms))
    assert rc == -4 and (tr == -5).all()   # DPG_ERR_SIZE
    assert ctx.icp_fetch_trace(2).shape == (3, 2, ms.value)
    ctx.close()


def test_checkpoint_rejects_foreign_files(tmp_path):
    """dpg_inc_load validates the file before it touches a device: a file that is not a graph
    checkpoint of this version (or is truncated) is rejected with DPG_ERR_ARG."""
    from dpgslam import api
    bad = tmp_path / "not_a_graph.bin"
    bad.write_bytes(b"DPGGRAPH" + b"\x07" * 200)
    with pytest.raises(_abi.DpgError, match="not a graph checkpoint"):
        api.IncGraph.load(None, str(bad))
    with pytest.raises(_abi.DpgError, match="cannot open"):
        api.IncGraph.load(None, str(tmp_path / "missing.bin"))


@pytest.mark.gpu
def test_gpu_checkpoint_resume_update_path(ctx, tmp_path):
    """dpg_inc_save / dpg_inc_load (SURVEY section 5 graph dump): a 300-node ISAM2 graph is saved,
    restored on a fresh context, and both continue with the same 150 updates -- the restored run
    agrees with the uninterrupted one to rounding (a fresh elimination order) and with the oracle;
    the relinearization schedule continues (update count restored: the 310th update relinearizes)."""
    from dpgslam import api
    X0, F = _sequence("config3", 450)
    key = _per_node(F)
    g = api.IncGraph(ctx, mode="isam2", reorder_every=64)
    o = O.OracleIncGraph(mode="isam2")
    for v in range(300):
        g.update(X0[v:v + 1], F[key == v])
        o.update(X0[v:v + 1], F[key == v])
    path = str(tmp_path / "graph.dpg")
    g.save(path)
    ctx2 = api.Context(0)
    h = api.IncGraph.load(ctx2, path)
    assert h.V == 300 and np.array_equal(h.poses(), g.poses())
    for v in range(300, 450):
        sg = g.update(X0[v:v + 1], F[key == v])
        sh = h.update(X0[v:v + 1], F[key == v])
        o.update(X0[v:v + 1], F[key == v])
        assert sg.relinearized == sh.relinearized and sg.n_factors == sh.n_factors
    assert np.abs(pose_diff(h.poses(), g.poses())).max() < 1e-9
    assert np.abs(pose_diff(h.poses(), o.poses())).max() < 1e-6
    h.close()
    g.close()
    ctx2.close()


@pytest.mark.gpu
def test_gpu_checkpoint_resume_add_node_path(tmp_path):
    """The checkpoint carries the scan store: a graph built node by node with dpg_add_node (the
    node's cloud, its successive alignment and loop closures by the reference rule) is saved at 60
    nodes, restored on a fresh context, and both add the same 40 nodes -- same alignments and
    factors, poses equal to rounding."""
    from dpgslam import api
    w = synth.generate("config3")
    p = _abi.default_icp_params()
    prior = np.zeros(1, _abi.FACTOR_DTYPE)
    prior["kind"], prior["i"], prior["info"] = _abi.DPG_FACTOR_PRIOR, 0, 1.0 / np.array([0.04, 0.04, 0.0225])
    ctx = api.Context(0)
    g = api.IncGraph(ctx, mode="isam2", reorder_every=16)
    passes = np.zeros(100, np.int32)
    for v in range(60):
        g.add_node(w.cloud(v), passes[:v + 1], w.est[v], extra=prior if v == 0 else None, icp_params=p)
    path = str(tmp_path / "graph_scans.dpg")
    g.save(path)
    ctx2 = api.Context(0)
    h = api.IncGraph.load(ctx2, path)
    assert h.V == 60 and np.array_equal(h.poses(), g.poses())
    for v in range(60, 100):
        sg = g.add_node(w.cloud(v), passes[:v + 1], w.est[v], icp_params=p)
        sh = h.add_node(w.cloud(v), passes[:v + 1], w.est[v], icp_params=p)
        assert (sg.n_icp_edges, sg.n_loop_closures) == (sh.n_icp_edges, sh.n_loop_closures)
        assert sg.update.n_factors == sh.update.n_factors
    assert np.abs(pose_diff(h.poses(), g.poses())).max() < 1e-9
    h.close()
    g.close()
    ctx2.close()
    ctx.close()


@pytest.mark.gpu
def test_gpu_checkpoint_failed_load_keeps_the_store(tmp_path):
    """A load that fails after the file was read (here: a multi-device context, which the incremental
    graph refuses) leaves the caller's scan store as it was -- its own 30 nodes, still aligned bit
    for bit as before (the store used to be replaced before the checks)."""
    from dpgslam import api
    w = synth.generate("config2")
    p = _abi.default_icp_params()
    ctx = api.Context(0)
    g = api.IncGraph(ctx, mode="isam2")
    prior = np.zeros(1, _abi.FACTOR_DTYPE)
    prior["kind"], prior["i"], prior["info"] = _abi.DPG_FACTOR_PRIOR, 0, 1.0 / np.array([0.04, 0.04, 0.0225])
    for v in range(12):
        g.add_node(w.cloud(v), np.zeros(v + 1, np.int32), w.est[v], extra=prior if v == 0 else None, icp_params=p)
    path = str(tmp_path / "graph12.dpg")
    g.save(path)
    g.close()
    ctx.close()
    V = 30
    with api.Context(0, virtual=2) as m:
        m.upload_scans(w.pts[:w.offsets[V]], w.offsets[:V + 1], p.downsample_icp_points_ratio)
        e = np.stack([np.arange(V - 1), np.arange(1, V)], 1).astype(np.int32)
        before, _ = m.icp_batch(e, w.est[:V], p, compute_cov=False)
        with pytest.raises(_abi.DpgError):
            api.IncGraph.load(m, path)
        after, _ = m.icp_batch(e, w.est[:V], p, compute_cov=False)
        assert before.tobytes() == after.tobytes()
