#!/usr/bin/env python3
"""Determinism of one angular ICP kernel variant: the same staged batch run R times (caller order),
every result compared with the first run's; reports the differing edges and fields.
usage: python tools/icp_det_check.py VARIANT [config] [runs]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpg-slam_amd"))
from dpgslam import _abi, api, synth  # noqa: E402

v = int(sys.argv[1])
cfg = sys.argv[2] if len(sys.argv) > 2 else "config4"
runs = int(sys.argv[3]) if len(sys.argv) > 3 else 6
w = synth.generate(cfg)
p = _abi.default_icp_params()
with api.Context(0) as ctx:
    ctx.set_icp_schedule("caller")
    ctx.set_icp_kernel_variant(v)
    ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
    ctx.icp_prepare(w.edges, w.est, p)
    ref = None
    for r in range(runs):
        ctx.icp_run(compute_cov=False)
        res, _ = ctx.icp_fetch(with_hessian=False)
        if ref is None:
            ref = res.copy()
            continue
        bad = np.nonzero([ref[e].tobytes() != res[e].tobytes() for e in range(len(res))])[0]
        print(f"run {r}: {len(bad)} edges differ from run 0")
        for e in bad[:4]:
            print("  edge", e, w.edges[e], "\n    run0", ref[e], "\n    now ", res[e])
            if os.environ.get("ORACLE"):   # which of the two is the oracle's (brute-force nn)?
                sys.path.insert(0, ROOT)
                from oracle import oracle
                o, _ = oracle.icp_batch(w.pts, w.offsets, w.edges[e:e + 1], w.est, p, nn=oracle.NN_BRUTE)
                print("    oracle", o[0], "run0 ==", o[0].tobytes() == ref[e].tobytes(),
                      "now ==", o[0].tobytes() == res[e].tobytes())
