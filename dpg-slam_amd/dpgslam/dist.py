"""Edge-sharded multi-GPU driver: one process per GPU, torch.distributed (RCCL over xGMI on the
"nccl" backend) for the single collective of the path.

  ICP:  edges are independent -> rank r aligns its share of the edges; no collective (every rank
        holds all scans).  The shares interleave the edge classes (edge_order): rank r takes the
        successive pairs r, r + N, ... and the loop closures r, r + N, ... -- successive pairs
        overlap more (more correspondences per iteration) and iterate longer, so the contiguous
        cost-balanced ranges of round 2 left them all to ranks 0-1.  The edge list and the ICP
        factor slots are permuted once so that every share stays one contiguous range.
  GN:   every rank holds the whole factor list (the sparsity pattern is global) but linearizes
        only its shard: rank 0 the prior + odometry factors and its ICP edges, rank r > 0 its ICP
        edges.  Per GN iteration ONE all-reduce(sum, fp64) of the packed [H upper | g | chi2]
        buffer, then every rank runs the identical supernodal Cholesky solve + retraction
        (replicated), so poses stay bitwise consistent without a broadcast.

The GN loop is written against a small backend protocol so the orchestration can be exercised on
CPU with the gloo backend (tests/test_dist_cpu.py); the GPU backend is `DeviceBackend`.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


def shard_ranges(n: int, world: int, weights: np.ndarray | None = None) -> list[tuple[int, int]]:
    """Contiguous ranges [b, e) covering [0, n), balanced by cumulative weight."""
    if world <= 1 or n == 0:
        return [(0, n)] + [(n, n)] * max(0, world - 1)
    w = np.ones(n) if weights is None else np.asarray(weights, np.float64)
    c = np.concatenate([[0.0], np.cumsum(w)])
    cuts = [0]
    for r in range(1, world):
        cuts.append(int(np.searchsorted(c, c[-1] * r / world, side="left")))
    cuts.append(n)
    cuts = np.maximum.accumulate(np.clip(cuts, 0, n))
    return [(int(cuts[r]), int(cuts[r + 1])) for r in range(world)]


def edge_order(world: int, n_edges: int, n_successive: int) -> tuple[np.ndarray, list[tuple[int, int]], list[int]]:
    """The interleaved shares: rank r gets successive pairs [r::world] then loop closures
    [r::world] (each in the caller's order: successive first, as they always become factors).
    Returns (perm, ranges, n_successive per rank): perm lists the edges rank 0's share first, and
    rank r's share is perm[ranges[r][0]:ranges[r][1]].  world 1: the identity."""
    succ, lc = np.arange(n_successive), np.arange(n_successive, n_edges)
    if world <= 1:
        return np.arange(n_edges), [(0, n_edges)], [n_successive]
    parts = [np.concatenate([succ[r::world], lc[r::world]]) for r in range(world)]
    cuts = np.concatenate([[0], np.cumsum([len(q) for q in parts])]).astype(int)
    return (np.concatenate(parts).astype(np.int64), [(int(cuts[r]), int(cuts[r + 1])) for r in range(world)],
            [len(succ[r::world]) for r in range(world)])


@dataclass
class ShardPlan:
    rank: int
    world: int
    edge_range: tuple[int, int]      # ICP edges of this rank: positions in `perm`
    factor_range: tuple[int, int]    # factors this rank linearizes (in the permuted factor list)
    n_always_local: int              # successive edges among this rank's edges (its first ones)
    perm: np.ndarray = None          # edge permutation (identity for world 1 / contiguous plans)

    def edges(self, edges: np.ndarray) -> np.ndarray:
        """This rank's edges, in dispatch order."""
        return edges[self.perm[self.edge_range[0]:self.edge_range[1]]]

    def factors(self, F: np.ndarray, icp_factor_first: int) -> np.ndarray:
        """The factor list with its ICP slots in permuted edge order (what every rank holds)."""
        G = F.copy()
        G[icp_factor_first:icp_factor_first + len(self.perm)] = F[icp_factor_first + self.perm]
        return G


def plan(rank: int, world: int, n_edges: int, n_successive: int, icp_factor_first: int,
         edge_cost: np.ndarray | None = None, strategy: str = "interleave") -> ShardPlan:
    """strategy "interleave" (default): edge_order's class-interleaved shares; "contiguous": round
    2's cost-balanced contiguous ranges of the caller's order (edge_cost weights)."""
    if strategy == "interleave":
        perm, ranges, n_succ = edge_order(world, n_edges, n_successive)
        er = ranges[rank]
        n_alw = n_succ[rank]
    else:
        perm = np.arange(n_edges)
        er = shard_ranges(n_edges, world, edge_cost)[rank]
        n_alw = int(np.clip(n_successive - er[0], 0, er[1] - er[0]))
    fb = 0 if rank == 0 else icp_factor_first + er[0]
    fe = icp_factor_first + er[1]
    return ShardPlan(rank, world, er, (fb, fe), n_alw, perm)


def check_convergence(rel_tol: float, abs_tol: float, cur: float, new: float) -> bool:
    """GTSAM checkConvergence with errorTol = 0 (NonlinearOptimizer.cpp)."""
    if new <= 0.0:
        return True
    dec = cur - new
    return (rel_tol != 0.0 and dec / cur <= rel_tol) or dec <= abs_tol


def gn_loop(backend, allreduce, params) -> dict:
    """Batch Gauss-Newton with one all-reduce per iteration (mirrors dpg_optimize_graph).

    backend: new_hb(), assemble(hb), chi2(hb) -> float, solve_retract(hb) (enqueue only),
             fetch(hb) -> (max|delta| of the last retraction, chi2 of hb, solver status)
    allreduce(hb): in-place sum over ranks (identity for one rank).
    Per iteration: solve + retract, re-linearize, all-reduce, then ONE read of the scalars."""
    hb = backend.new_hb()
    backend.assemble(hb)
    allreduce(hb)
    cur = backend.chi2(hb)
    stats = {"iterations": 0, "pcg_iterations": 0, "initial_error": cur, "final_error": cur, "last_delta_inf": 0.0}
    if cur <= 0.0 or params.max_iterations <= 0:
        return stats
    it = 0
    while True:
        backend.solve_retract(hb)
        it += 1
        backend.assemble(hb)
        allreduce(hb)
        dinf, new, status = backend.fetch(hb)
        if status != 0:
            raise RuntimeError(f"linear solve failed (status {status}): H not positive definite")
        stats.update(iterations=it, final_error=new, last_delta_inf=dinf)
        if it >= params.max_iterations:
            break
        if params.use_error_criteria:
            if check_convergence(params.relative_error_tol, params.absolute_error_tol, cur, new) or not np.isfinite(cur):
                break
        elif dinf < params.delta_tol:
            break
        cur = new
    return stats


class DeviceBackend:
    """GN backend on one GPU: libdpg step API + a torch-owned packed buffer (so torch.distributed
    can all-reduce it in place with RCCL)."""

    def __init__(self, ctx, hb_size: int, chi2_index: int, device):
        import torch
        self.ctx = ctx
        self.n = hb_size
        self.chi2_index = chi2_index
        self.device = device
        self.torch = torch

    def new_hb(self):
        return self.torch.zeros(self.n, dtype=self.torch.float64, device=self.device)

    def assemble(self, hb):
        self.ctx.gn_assemble(hb.data_ptr())

    def chi2(self, hb) -> float:
        return float(hb[self.chi2_index].item())

    def solve_retract(self, hb):
        self.ctx.gn_solve_retract_async(hb.data_ptr())

    def fetch(self, hb):
        return self.ctx.gn_fetch(hb.data_ptr())


class HostCollective:
    """libdpg's rank form over a torch.distributed process group instead of RCCL
    (dpg_ctx_create_rank_ops): the three blocking host-memory collectives of dpg_coll_ops -- the
    cost all-reduce of the LPT plan, the results' all-gather, the packed system's all-reduce per
    Gauss-Newton iteration -- as gloo calls.  The world > 1 rank form then runs where RCCL cannot
    (several ranks on one card); `calls` counts what each rank issued (they must agree)."""

    def __init__(self, group=None):
        import ctypes as C
        import torch
        import torch.distributed as dist
        from . import _abi
        self.group, self.dist, self.torch, self.C = group, dist, torch, C
        self.world = dist.get_world_size(group)
        self.calls = {"allreduce_f64": 0, "allreduce_f32": 0, "allgather": 0}
        self.error = None
        # the C side keeps the function pointers: these thunks live as long as this object
        self._f64 = _abi.ALLREDUCE_F64(self._allreduce_f64)
        self._f32 = _abi.ALLREDUCE_F32(self._allreduce_f32)
        self._ag = _abi.ALLGATHER(self._allgather)
        self.ops = _abi.CollOps(None, self._f64, self._f32, self._ag)

    def _guard(self, fn):
        try:
            fn()
            return 0
        except Exception as e:   # reported to libdpg as a failed collective
            self.error = e
            return 1

    def _allreduce(self, buf, n, dtype, key):
        def run():
            a = np.ctypeslib.as_array(buf, shape=(int(n),))
            t = self.torch.from_numpy(a)          # shares the C buffer: summed in place
            self.dist.all_reduce(t, group=self.group)
            self.calls[key] += 1
        return self._guard(run)

    def _allreduce_f64(self, user, buf, n):
        return self._allreduce(buf, n, np.float64, "allreduce_f64")

    def _allreduce_f32(self, user, buf, n):
        return self._allreduce(buf, n, np.float32, "allreduce_f32")

    def _allgather(self, user, send, recv, nbytes):
        def run():
            nb = int(nbytes)
            src = np.ctypeslib.as_array(self.C.cast(send, self.C.POINTER(self.C.c_uint8)), shape=(nb,))
            dst = np.ctypeslib.as_array(self.C.cast(recv, self.C.POINTER(self.C.c_uint8)), shape=(nb * self.world,))
            outs = [self.torch.empty(nb, dtype=self.torch.uint8) for _ in range(self.world)]
            self.dist.all_gather(outs, self.torch.from_numpy(src.copy()), group=self.group)
            for r, o in enumerate(outs):
                dst[r * nb:(r + 1) * nb] = o.numpy()
            self.calls["allgather"] += 1
        return self._guard(run)
