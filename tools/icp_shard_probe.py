"""Probe: the ICP kernel on each rank's share of config 4 at N = 2, 4, 8 (dpgslam.dist.plan, one
rank's edges at a time on this one GPU), for the round-2 contiguous cost-balanced ranges and the
class-interleaved shares, optionally with the kernel's wave-priority aging (DPG_ICP_PRIO_AGE).
No measured iteration counts are used for the shares or their order.
usage: python tools/icp_shard_probe.py [strategy:age ...]   (default contiguous:0 interleave:0 interleave:16)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpg-slam_amd")]
import numpy as np  # noqa: E402

from dpgslam import _abi, api, synth  # noqa: E402
from dpgslam import dist as D  # noqa: E402

modes = sys.argv[1:] or ["contiguous:0", "interleave:0", "interleave:16"]
w = synth.generate("config4")
p = _abi.default_icp_params()
ctx = api.Context(0)
ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)


def run(edges, reps=3):
    ms = []
    for _ in range(reps):
        ctx.icp_batch(edges, w.est, p, compute_cov=False)
        ms.append(ctx.icp_kernel_ms())
    return float(np.median(ms))


run(w.edges)   # warm-up
n_src = np.diff(w.offsets)[w.edges[:, 1]]
n_tgt = np.diff(w.offsets)[w.edges[:, 0]]
for mode in modes:
    strategy, _, age = mode.partition(":")
    os.environ["DPG_ICP_PRIO_AGE"] = age or "0"
    full_ms = run(w.edges)
    print(f"[{mode}] all {w.E} edges: {full_ms:.3f} ms", flush=True)
    for world in (2, 4, 8):
        times = []
        for rank in range(world):
            pl = D.plan(rank, world, w.E, w.n_successive, w.icp_factor_first, edge_cost=n_src * n_tgt, strategy=strategy)
            times.append(run(pl.edges(w.edges)))
        print(f"[{mode}] N={world}: per rank " + " ".join(f"{t:.3f}" for t in times) +
              f"  slowest {max(times):.3f} ms (1/N of all: {full_ms / world:.3f} ms)", flush=True)
