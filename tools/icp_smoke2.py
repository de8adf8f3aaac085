#!/usr/bin/env python3
"""Config-2 batched ICP vs the oracle at one defer cap (bit-exact), printing as it goes.
usage: python tools/icp_smoke2.py CAP"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dpg-slam_amd"))
from dpgslam import _abi, api, synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

cap = int(sys.argv[1])
w = synth.generate("config2")
p = _abi.default_icp_params()
print(f"cap {cap}: generated config2 E={w.E}", flush=True)
with api.Context(0) as ctx:
    ctx.set_icp_defer_cap(cap)
    ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
    t = time.time()
    res, _ = ctx.icp_batch(w.edges, w.est, p, compute_cov=False)
    print(f"cap {cap}: GPU batch {time.time() - t:.2f} s, status counts {np.bincount(res['status'])}", flush=True)
ref, _ = O.icp_batch(w.pts, w.offsets, w.edges, w.est, p, O.NN_GRID, 8)
same = res.tobytes() == np.asarray(ref).tobytes()
print(f"cap {cap}: bit-exact vs oracle: {same}", flush=True)
sys.exit(0 if same else 1)
