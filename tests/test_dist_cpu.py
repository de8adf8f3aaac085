"""Multi-rank orchestration on CPU (gloo, world_size 2): edge/factor sharding and the one
all-reduce per GN iteration of dpgslam.dist.  The per-rank linear algebra here is a dense numpy
stand-in built from the ORACLE's factor linearization (test infrastructure); on GPUs the same
gn_loop drives libdpg through DeviceBackend and RCCL."""
import os
import socket

import numpy as np
import pytest

from graphs import gtsam_test_graph, pose_diff


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class DenseBackend:
    """Dense H of the factors in [fb, fe), solved with numpy (test stand-in)."""

    def __init__(self, X0, F, fr):
        import torch
        from oracle import oracle as O
        self.torch, self.O = torch, O
        self.X = np.array(X0, float)
        self.F, self.fr = F, fr
        self.n = 3 * len(X0)

    def new_hb(self):
        return self.torch.zeros(self.n * self.n + self.n + 2, dtype=self.torch.float64)

    def assemble(self, hb):
        H, g, chi2 = np.zeros((self.n, self.n)), np.zeros(self.n), 0.0
        for k in range(*self.fr):
            f = self.F[k]
            e, Ai, Aj = self.O.linearize(f, self.X)
            W = np.diag(f["info"])
            i = 3 * f["i"]
            chi2 += 0.5 * e @ W @ e
            H[i:i + 3, i:i + 3] += Ai.T @ W @ Ai
            g[i:i + 3] += Ai.T @ W @ e
            if f["kind"] == 1:
                j = 3 * f["j"]
                H[j:j + 3, j:j + 3] += Aj.T @ W @ Aj
                H[i:i + 3, j:j + 3] += Ai.T @ W @ Aj
                H[j:j + 3, i:i + 3] += Aj.T @ W @ Ai
                g[j:j + 3] += Aj.T @ W @ e
        hb[: self.n * self.n] = self.torch.from_numpy(H.ravel())
        hb[self.n * self.n: self.n * self.n + self.n] = self.torch.from_numpy(g)
        hb[-2] = chi2

    def chi2(self, hb):
        return float(hb[-2])

    def solve_retract(self, hb):
        H = hb[: self.n * self.n].numpy().reshape(self.n, self.n)
        g = hb[self.n * self.n: self.n * self.n + self.n].numpy()
        d = np.linalg.solve(H, -g).reshape(-1, 3)
        for v in range(len(self.X)):
            c, s = np.cos(self.X[v, 2]), np.sin(self.X[v, 2])
            self.X[v, 0] += c * d[v, 0] - s * d[v, 1]
            self.X[v, 1] += s * d[v, 0] + c * d[v, 1]
            th = self.X[v, 2] + d[v, 2]
            self.X[v, 2] = np.arctan2(np.sin(th), np.cos(th))
        self.last_dinf = float(np.abs(d).max())

    def fetch(self, hb):
        return self.last_dinf, self.chi2(hb), 0


def _worker(rank, world, port, X0, F, nb_first, out):
    import torch.distributed as dist
    from dpgslam import _abi
    from dpgslam import dist as D
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    n_icp = len(F) - nb_first
    pl = D.plan(rank, world, n_icp, n_successive=0, icp_factor_first=nb_first)
    be = DenseBackend(X0, pl.factors(F, nb_first), pl.factor_range)
    gp = _abi.default_gn_params()
    st = D.gn_loop(be, lambda hb: dist.all_reduce(hb), gp)
    out[rank] = (be.X.copy(), st["iterations"], pl.factor_range)
    dist.destroy_process_group()


def _run(world, X0, F, nb_first):
    import torch.multiprocessing as mp
    mgr = mp.Manager()
    out = mgr.dict()
    port = _free_port()
    mp.spawn(_worker, args=(world, port, X0, F, nb_first, out), nprocs=world, join=True)
    return dict(out)


def _random_graph(V=40, seed=7):
    from dpgslam import api
    rng = np.random.default_rng(seed)
    gt = np.cumsum(np.c_[np.ones(V), rng.normal(0, 0.3, V), rng.normal(0, 0.2, V)], 0)
    gt[:, 2] = np.arctan2(np.sin(gt[:, 2]), np.cos(gt[:, 2]))
    from dpgslam.synth import _relative
    fs = [api.prior_factor(0, tuple(gt[0]), (0.2, 0.2, 0.15))]
    pairs = [(i, i + 1) for i in range(V - 1)] + [(i, i + k) for k in (3, 7) for i in range(0, V - k, 2)]
    for i, j in pairs:
        z = _relative(gt[j], gt[i]) + rng.normal(0, [0.05, 0.05, 0.01])
        fs.append(api.between_factor(i, j, z, (0.1, 0.1, 0.05)))
    X0 = gt + rng.normal(0, [0.2, 0.2, 0.05], gt.shape)
    return X0, np.concatenate(fs)


@pytest.mark.parametrize("graph", ["gtsam_test", "random40"])
def test_world2_matches_world1_and_oracle(graph):
    from oracle import oracle as O
    if graph == "gtsam_test":
        X0, F, _ = gtsam_test_graph()
    else:
        X0, F = _random_graph()
    r1 = _run(1, X0, F, 1)
    r2 = _run(2, X0, F, 1)
    Xo, _ = O.optimize_graph(X0, F)
    assert r2[0][2][0] == 0 and r2[0][2][1] == r2[1][2][0] and r2[1][2][1] == len(F), "factor shards must tile"
    np.testing.assert_array_equal(r2[0][0], r2[1][0])        # replicated solve: ranks agree bitwise
    assert np.abs(pose_diff(r2[0][0], r1[0][0])).max() < 1e-9
    assert np.abs(pose_diff(r1[0][0], Xo)).max() < 1e-9


def test_shard_ranges_tile_and_balance():
    from dpgslam.dist import plan, shard_ranges
    for n, w in [(0, 2), (1, 4), (10, 3), (20000, 8), (20000, 1)]:
        rs = shard_ranges(n, w)
        assert len(rs) == w and rs[0][0] == 0 and rs[-1][1] == n
        assert all(rs[k][1] == rs[k + 1][0] for k in range(w - 1))
        if n >= w:
            sz = [e - b for b, e in rs]
            assert max(sz) - min(sz) <= 1
    cost = np.r_[np.full(100, 10.0), np.ones(900)]
    rs = shard_ranges(1000, 2, cost)
    assert abs(cost[rs[0][0]:rs[0][1]].sum() - cost[rs[1][0]:rs[1][1]].sum()) <= 10.0
    # ICP factor ownership: successive edges stay "always kept" wherever they land
    for strategy in ("contiguous", "interleave"):
        p0, p1 = plan(0, 2, 20000, 4999, 5000, strategy=strategy), plan(1, 2, 20000, 4999, 5000, strategy=strategy)
        assert p0.factor_range[0] == 0 and p0.factor_range[1] == p1.factor_range[0] and p1.factor_range[1] == 25000
        assert p0.n_always_local + p1.n_always_local == 4999


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_interleaved_shares(world):
    """dist.edge_order: a permutation; every rank's share is one contiguous range of it, its
    successive pairs first (the always-kept factors), each class spread evenly over the ranks; the
    permuted factor list keeps every base factor and moves each ICP slot with its edge."""
    from dpgslam.dist import plan
    E, ns, first = 20000, 4999, 5000
    plans = [plan(r, world, E, ns, first) for r in range(world)]
    perm = plans[0].perm
    assert np.array_equal(np.sort(perm), np.arange(E))
    assert plans[0].edge_range[0] == 0 and plans[-1].edge_range[1] == E
    for r, pl in enumerate(plans):
        a, b = pl.edge_range
        share = perm[a:b]
        k = pl.n_always_local
        assert np.all(share[:k] < ns) and np.all(share[k:] >= ns)
        assert np.array_equal(share[:k], np.arange(r, ns, world))
        assert np.array_equal(share[k:], np.arange(ns + r, E, world))
        if r + 1 < world:
            assert pl.edge_range[1] == plans[r + 1].edge_range[0]
    F = np.zeros(first + E, [("i", np.int32), ("j", np.int32)])
    F["i"], F["j"] = np.arange(first + E), -1
    G = plans[0].factors(F, first)
    assert np.array_equal(G["i"][:first], np.arange(first)) and np.array_equal(G["i"][first:], first + perm)


def _lpt_reference(cost, world):
    """longest-processing-time, restated: edges by cost descending (stable), each to the rank with
    the least load so far (lowest rank among equals)."""
    order = sorted(range(len(cost)), key=lambda e: -float(np.float32(cost[e])))
    load = [0.0] * world
    owner = [0] * len(cost)
    disp = [[] for _ in range(world)]
    for e in order:
        r = min(range(world), key=lambda q: (load[q], q))
        owner[e] = r
        load[r] += float(np.float32(cost[e]))
        disp[r].append(e)
    return owner, disp


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("measured", [False, True])
def test_shard_plan_and_rank_form_gather(world, measured):
    """dpg_shard_plan / dpg_shard_reassemble (libdpg host code, no GPU): the assignment equals the
    restated LPT (or e mod world), every rank's dispatch list covers its edges, and the rank form's
    all-gather -- each rank's results in its local order (its edges ascending, as stage_device
    numbers them), padded to the largest share -- comes back in the caller's order, record for record
    (the rank form's reassembly was only reachable with world > 1 on GPUs)."""
    from dpgslam import api
    rng = np.random.default_rng(world * 10 + measured)
    ne = 997
    cost = (rng.integers(1, 60, ne) * rng.integers(200, 1200, ne)).astype(np.float32) if measured else None
    if measured:
        cost[::50] = cost[1]   # ties: lower index first
    owner, disp, counts = api.shard_plan(ne, world, cost)
    if measured:
        ro, rd = _lpt_reference(cost, world)
        assert owner.tolist() == ro
        assert np.concatenate([np.asarray(d, np.int64) for d in rd]).tolist() == disp.tolist()
    else:
        assert np.array_equal(owner, np.arange(ne) % world)
    assert counts.sum() == ne and np.array_equal(np.sort(disp), np.arange(ne))
    first = np.r_[0, np.cumsum(counts)]
    rec = 24
    slice_ = int(max(counts.max(), 1))
    gathered = np.zeros((world, slice_, rec), np.uint8)
    for r in range(world):
        mine = disp[first[r]:first[r + 1]]
        assert np.all(owner[mine] == r)
        local = np.sort(mine)                                # result j of rank r is edge local[j]
        for j, e in enumerate(local):
            gathered[r, j] = np.frombuffer(np.array([e, e * 7 + r, -e], np.int64).tobytes(), np.uint8)
    out = api.shard_reassemble(owner, world, slice_, gathered.reshape(-1), rec).view(np.int64).reshape(ne, 3)
    assert np.array_equal(out[:, 0], np.arange(ne)) and np.array_equal(out[:, 1], np.arange(ne) * 7 + owner)


def _coll_worker(rank, world, port, out):
    import ctypes as C
    import torch.distributed as dist
    from dpgslam import dist as D
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    coll = D.HostCollective()
    a = np.arange(5, dtype=np.float64) * (rank + 1)
    f = np.full(3, rank + 0.5, np.float32)
    send = np.frombuffer(bytes([rank] * 7), np.uint8).copy()
    recv = np.zeros(7 * world, np.uint8)
    rc = [coll.ops.allreduce_sum_f64(None, a.ctypes.data_as(C.POINTER(C.c_double)), 5),
          coll.ops.allreduce_sum_f32(None, f.ctypes.data_as(C.POINTER(C.c_float)), 3),
          coll.ops.allgather(None, send.ctypes.data, recv.ctypes.data, 7)]
    out[rank] = (rc, a.copy(), f.copy(), recv.copy(), dict(coll.calls))
    dist.destroy_process_group()


def test_host_collective_over_gloo():
    """dist.HostCollective -- the dpg_coll_ops callbacks libdpg's rank form calls through
    dpg_ctx_create_rank_ops -- sums in place and gathers in rank order over gloo (world 2)."""
    import torch.multiprocessing as mp
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_coll_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        rc, a, f, recv, calls = out[r]
        assert rc == [0, 0, 0]
        assert np.array_equal(a, np.arange(5) * 3.0) and np.array_equal(f, np.full(3, 2.0, np.float32))
        assert recv.tolist() == [0] * 7 + [1] * 7
        assert calls == {"allreduce_f64": 1, "allreduce_f32": 1, "allgather": 1}
