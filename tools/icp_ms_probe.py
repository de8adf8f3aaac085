#!/usr/bin/env python3
"""Why the bench's ICP kernel time differs from the A/B tool's: the same staged config-4 batch
timed (HIP events, dpg_icp_kernel_ms) alone without / with the covariance, and inside the bench's
full step (ICP + covariance + GN), both dispatch schedules, in one process.
usage: python tools/icp_ms_probe.py [rounds]"""
import os
import sys

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

    def full(cov):
        ctx.icp_run(compute_cov=cov)
        ctx.gn_take_icp(w.icp_factor_first, w.E, w.n_successive, p)
        ctx.gn_set_poses(X0)
        ctx.gn_run()

    forms = {"icp": lambda: ctx.icp_run(compute_cov=False), "icp+cov": lambda: ctx.icp_run(compute_cov=True),
             "step": lambda: full(True), "step-nocov": lambda: full(False)}
    for sched in ("caller", "measured"):
        ctx.set_icp_schedule(sched)
        ms = {k: [] for k in forms}
        for r in range(rounds + 1):
            for k, f in forms.items():
                f()
                ctx.synchronize()
                if r > 0:
                    ms[k].append(ctx.icp_kernel_ms())
        for k, v in ms.items():
            print(f"{sched:9s} {k:11s} icp kernel median {np.median(v):.3f} ms  min {np.min(v):.3f}")
