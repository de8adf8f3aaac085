#!/usr/bin/env python3
"""A/B of the angular ICP kernel's cooperative-queue threshold (dpg_ctx_set_icp_defer_cap) on a
config's batched ICP, interleaved rounds in ONE process (cdna_hip_programming.md rule 24).  Every
variant must give byte-identical results to the first one listed.
usage: python tools/icp_cap_ab.py [caps...] (default 256 64); ICP_CONFIG (config4), AB_ROUNDS (5)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpg-slam_amd"))
from dpgslam import _abi, api, synth  # noqa: E402

variants = sys.argv[1:] or ["256", "64"]
rounds = int(os.environ.get("AB_ROUNDS", "5"))
w = synth.generate(os.environ.get("ICP_CONFIG", "config4"))
p = _abi.default_icp_params()
ms = {v: [] for v in variants}
with api.Context(0) as ctx:
    ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
    ctx.icp_prepare(w.edges, w.est, p)
    ref = None
    for r in range(rounds + 1):
        for v in variants:
            ctx.set_icp_defer_cap(int(v))
            ctx.icp_run(compute_cov=False)
            ctx.synchronize()
            k = ctx.icp_kernel_ms()
            res, _ = ctx.icp_fetch(with_hessian=False)
            b = res.tobytes()
            if ref is None:
                ref = b
            assert b == ref, f"cap {v}: results differ from variant {variants[0]}"
            if r > 0:
                ms[v].append(k)
for v in variants:
    a = np.array(ms[v])
    print(f"cap {v}: icp kernel median {np.median(a):.3f} ms  min {a.min():.3f}  (rounds {len(a)})")
print("all results byte-identical")
