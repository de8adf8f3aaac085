"""Probe: does the ORDER of the edges in one batched ICP launch change the kernel time (tail effect
of long alignments dispatched last)?  Runs config 4's 20 000 edges in the natural order, in
descending order of their (measured) iteration counts, in random order, and in descending order
of a cheap a-priori proxy (the loop-closure distance / guess), reporting kernel ms for each."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpg-slam_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from dpgslam import _abi, api, synth  # noqa: E402

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


run(w.edges)   # warm-up (the first launch pays for cold caches)
base_ms, res = run(w.edges)
it = res["iterations"].astype(np.int64)
print(f"natural: {base_ms:.3f} ms; iterations mean {it.mean():.1f} max {it.max()} p99 {np.percentile(it, 99):.0f}")
order = np.argsort(-it, kind="stable")
ms, r2 = run(w.edges[order])
assert np.array_equal(r2["iterations"], it[order])
print(f"desc iterations: {ms:.3f} ms")
rng = np.random.default_rng(0)
ms, _ = run(w.edges[rng.permutation(len(w.edges))])
print(f"random: {ms:.3f} ms")
d = w.est[w.edges[:, 1], :2] - w.est[w.edges[:, 0], :2]
proxy = np.hypot(d[:, 0], d[:, 1]) + 2.0 * np.abs(np.angle(np.exp(1j * (w.est[w.edges[:, 1], 2] - w.est[w.edges[:, 0], 2]))))
ms, _ = run(w.edges[np.argsort(-proxy, kind="stable")])
print(f"desc proxy: {ms:.3f} ms (corr proxy/iters {np.corrcoef(proxy, it)[0, 1]:.2f})")
