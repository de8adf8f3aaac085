#!/usr/bin/env python3
"""Where two angular ICP kernel variants first differ: per-edge results and the per-iteration
correspondence trace of the first differing edge (config 2, the first EDGES edges).
usage: python tools/icp_var_diff.py VA VB [config] [edges]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpg-slam_amd"))
from dpgslam import _abi, api, synth  # noqa: E402

va, vb = int(sys.argv[1]), int(sys.argv[2])
cfg = sys.argv[3] if len(sys.argv) > 3 else "config2"
ne = int(sys.argv[4]) if len(sys.argv) > 4 else 200
w = synth.generate(cfg)
p = _abi.default_icp_params()
E = w.edges[:ne]
out = {}
with api.Context(0) as ctx:
    ctx.set_icp_schedule(os.environ.get("SCHED", "caller"))
    ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
    full = {}
    for v in (va, vb):   # all edges without the trace, then the trace of the first differing ones
        ctx.set_icp_kernel_variant(v)
        full[v], _ = ctx.icp_batch(E, w.est, p, compute_cov=False)   # (measured: planned from the last run)
    bad = [e for e in range(len(E)) if full[va][e].tobytes() != full[vb][e].tobytes()]
    print(f"{len(bad)} of {len(E)} edges differ")
    E = E[bad[:5]]
    for v in (va, vb):
        ctx.set_icp_kernel_variant(v)
        res, _ = ctx.icp_batch(E, w.est, p, compute_cov=False, trace_iters=60)
        out[v] = (res, ctx.icp_fetch_trace(60))
ra, ta = out[va]
rb, tb = out[vb]
print("traced edges:", bad[:5], [ra[e].tobytes() != rb[e].tobytes() for e in range(len(E))])
for e in range(len(E)):
    print("edge", e, "A", ra[e], "\n       B", rb[e])
    d = np.nonzero((ta[e] != tb[e]).any(1))[0]
    if len(d):
        k = d[0]
        pts = np.nonzero(ta[e, k] != tb[e, k])[0]
        print(f"  first differing iteration {k}: points {pts[:10]} A {ta[e, k, pts[:10]]} B {tb[e, k, pts[:10]]}")
    else:
        print("  traces equal")
