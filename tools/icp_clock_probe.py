#!/usr/bin/env python3
"""Does the ICP kernel's time depend on what ran before it (clock ramp after a latency-bound GN
phase)?  The same staged config-4 batch timed (HIP events) right after another ICP launch, after a
GN solve of the graph, and after the GPU sat idle for 4 / 50 ms, interleaved in one process.
usage: python tools/icp_clock_probe.py [rounds]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpg-slam_amd"))
from dpgslam import _abi, api, synth  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 8
w = synth.generate("config4")
p = _abi.default_icp_params()
gp = _abi.default_gn_params()
X0 = w.est.astype(np.float64)
with api.Context(0) as ctx:
    ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
    ctx.icp_prepare(w.edges, w.est, p)
    ctx.gn_setup(w.V, w.factors_placeholder(), params=gp)
    ctx.icp_run(compute_cov=False)
    ctx.gn_take_icp(w.icp_factor_first, w.E, w.n_successive, p)

    def gn():
        ctx.gn_set_poses(X0)
        ctx.gn_run()

    pre = {"after-icp": lambda: ctx.icp_run(compute_cov=False), "after-gn": gn,
           "after-idle-4ms": lambda: time.sleep(0.004), "after-idle-50ms": lambda: time.sleep(0.05)}
    ms = {k: [] for k in pre}
    for r in range(rounds + 1):
        for k, f in pre.items():
            f()   # no synchronisation: the ICP is queued behind it, as in the bench step
            ctx.icp_run(compute_cov=False)
            ctx.synchronize()
            if r > 0:
                ms[k].append(ctx.icp_kernel_ms())
    for k, v in ms.items():
        print(f"{k:16s} icp kernel median {np.median(v):.3f} ms  min {np.min(v):.3f}  max {np.max(v):.3f}")
