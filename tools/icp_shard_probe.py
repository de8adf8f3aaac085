"""Probe: the ICP kernel on ONE rank's shard of config 4 at N = 2, 4, 8 (bench.py's cost-balanced
contiguous edge ranges, dpgslam.dist.plan), in the natural order and in descending order of the
measured iteration counts (the ideal longest-first dispatch) -- how much of a shard's kernel time is
the tail of long alignments dispatched last, where fewer edges per workgroup slot remain.
usage: python tools/icp_shard_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpg-slam_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from dpgslam import _abi, api, synth  # noqa: E402
from dpgslam import dist as D  # noqa: E402

w = synth.generate("config4")
p = _abi.default_icp_params()
ctx = api.Context(0)
ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)


def run(edges, reps=3):
    ms = []
    for _ in range(reps):
        res, _ = ctx.icp_batch(edges, w.est, p, compute_cov=False)
        ms.append(ctx.icp_kernel_ms())
    return float(np.median(ms)), res


run(w.edges)   # warm-up
full_ms, res = run(w.edges)
it_all = res["iterations"].astype(np.int64)
print(f"all 20000 edges: {full_ms:.3f} ms", flush=True)
n_src = np.diff(w.offsets)[w.edges[:, 1]]
n_tgt = np.diff(w.offsets)[w.edges[:, 0]]
for world in (2, 4, 8):
    worst_nat, worst_desc = 0.0, 0.0
    for rank in range(world):
        e0, e1 = D.plan(rank, world, w.E, w.n_successive, w.icp_factor_first, edge_cost=n_src * n_tgt).edge_range
        sub = w.edges[e0:e1]
        nat, _ = run(sub)
        order = np.argsort(-it_all[e0:e1], kind="stable")
        desc, _ = run(sub[order])
        worst_nat, worst_desc = max(worst_nat, nat), max(worst_desc, desc)
        print(f"N={world} rank {rank}: {e1 - e0} edges, natural {nat:.3f} ms, longest-first {desc:.3f} ms", flush=True)
    print(f"N={world}: slowest rank natural {worst_nat:.3f} ms, longest-first {worst_desc:.3f} ms "
          f"(ideal 1/N of all: {full_ms / world:.3f} ms)", flush=True)
