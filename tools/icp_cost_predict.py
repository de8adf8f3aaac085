#!/usr/bin/env python3
"""How predictable is an alignment's cost before it runs?  (VERDICT r2 "balance the ICP shards with
an a-priori cost proxy".)  Runs config 4's batched ICP once on the GPU, then relates the measured
iteration counts (cost = iterations x source points) to what is known before the alignment: the
edge class (successive / loop closure), the guess's translation and rotation (R3), the cloud sizes
and the node separation.  Prints correlations and the R^2 of a least-squares fit.
usage: python tools/icp_cost_predict.py [config]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpg-slam_amd")]
import numpy as np  # noqa: E402

from dpgslam import _abi, api, synth  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "config4"
w = synth.generate(name)
p = _abi.default_icp_params()
with api.Context(0) as ctx:
    ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
    res, _ = ctx.icp_batch(w.edges, w.est, p, compute_cov=False)
it = res["iterations"].astype(np.float64)
E, ns = w.E, w.n_successive
cnt = (np.diff(w.offsets) + p.downsample_icp_points_ratio - 1) // p.downsample_icp_points_ratio
N = cnt[w.edges[:, 1]].astype(np.float64)
M = cnt[w.edges[:, 0]].astype(np.float64)
rel = w.est[w.edges[:, 1]] - w.est[w.edges[:, 0]]   # source minus target estimate (map frame)
tr = np.hypot(rel[:, 0], rel[:, 1])
rot = np.abs((rel[:, 2] + np.pi) % (2 * np.pi) - np.pi)
sep = np.log1p(np.abs(w.edges[:, 0] - w.edges[:, 1]).astype(np.float64))
cls = (np.arange(E) >= ns).astype(np.float64)
cost = it * N
print(f"{name}: {E} edges; iterations mean {it.mean():.2f} (successive {it[:ns].mean():.2f}, loop closures "
      f"{it[ns:].mean():.2f}), p50 {np.median(it):.0f}, p99 {np.percentile(it, 99):.0f}, max {it.max():.0f}")
print(f"cost = iterations x source points: coefficient of variation {cost.std() / cost.mean():.3f}")
feats = {"class": cls, "guess translation": tr, "guess rotation": rot, "source points": N, "N x M": N * M,
         "log node separation": sep}
for k, f in feats.items():
    print(f"  corr({k:20s}, iterations) = {np.corrcoef(f, it)[0, 1]:+.3f}   corr(., cost) = {np.corrcoef(f, cost)[0, 1]:+.3f}")
X = np.stack([np.ones(E)] + list(feats.values()) + [tr * cls, rot * cls], 1)
for tgt, y in (("iterations", it), ("cost", cost)):
    coef, *_ = np.linalg.lstsq(X, y, rcond=None)
    r2 = 1 - ((y - X @ coef) ** 2).sum() / ((y - y.mean()) ** 2).sum()
    print(f"least-squares fit of {tgt} on all features: R^2 = {r2:.4f}")
