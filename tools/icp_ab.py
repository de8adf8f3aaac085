#!/usr/bin/env python3
"""A/B of the angular ICP kernel's cooperative-queue threshold on config 4, interleaved rounds in
ONE process (cdna_hip_programming.md rule 24).  Every setting must give byte-identical results to
the in-lane-only run (cap 0).  usage: python tools/icp_ab.py [caps...] (default 0 16 32 64 128)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpg-slam_amd"))
from dpgslam import _abi, api, synth  # noqa: E402

caps = [int(a) for a in sys.argv[1:]] or [0, 16, 32, 64, 128]
rounds = int(os.environ.get("AB_ROUNDS", "5"))
w = synth.generate("config4")
p = _abi.default_icp_params()
ms = {c: [] for c in caps}
with api.Context(0) as ctx:
    ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
    ctx.icp_prepare(w.edges, w.est, p)
    ref = None
    for r in range(rounds + 1):
        for c in caps:
            ctx.set_icp_defer_cap(c)
            ctx.icp_run(compute_cov=False)
            ctx.synchronize()
            k = ctx.icp_kernel_ms()
            res, _ = ctx.icp_fetch(with_hessian=False)
            b = res.tobytes()
            if ref is None:
                ref = b
            assert b == ref, f"cap {c}: results differ from the first run"
            if r > 0:
                ms[c].append(k)
for c in caps:
    a = np.array(ms[c])
    print(f"defer_cap {c:4d}: icp kernel median {np.median(a):.3f} ms  min {a.min():.3f}  (rounds {len(a)})")
print("all results byte-identical")
