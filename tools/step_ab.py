#!/usr/bin/env python3
"""A/B of a context setting on the bench step (config 4: ICP of all edges + covariance + factors on
the device + GN to convergence), interleaved rounds in ONE process; the step's wall time, the ICP
kernel and the GN share as bench.py computes them.  Every setting must reach the same final error.
usage: python tools/step_ab.py SETTING v1 v2 ...   SETTING: cov_workgroups | defer_cap
       AB_ROUNDS (6), AB_STEPS (5)"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpg-slam_amd"))
from dpgslam import _abi, api, synth  # noqa: E402

setting, vals = sys.argv[1], [int(v) for v in sys.argv[2:]]
rounds, steps = int(os.environ.get("AB_ROUNDS", "6")), int(os.environ.get("AB_STEPS", "5"))
w = synth.generate("config4")
p = _abi.default_icp_params()
gp = _abi.default_gn_params()
X0 = w.est.astype(np.float64)
with api.Context(0) as ctx:
    ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
    ctx.icp_prepare(w.edges, w.est, p)
    ctx.gn_setup(w.V, w.factors_placeholder(), params=gp)
    apply = {"cov_workgroups": ctx.set_cov_workgroups, "defer_cap": ctx.set_icp_defer_cap}[setting]

    def step():
        ctx.icp_run(compute_cov=True)
        ctx.gn_take_icp(w.icp_factor_first, w.E, w.n_successive, p)
        ctx.gn_set_poses(X0)
        return ctx.gn_run()[0]

    out = {v: {"step": [], "icp": [], "gn": []} for v in vals}
    err = {}
    for r in range(rounds + 1):
        for v in vals:
            apply(v)
            step()
            ctx.synchronize()
            for _ in range(steps):
                t0 = time.perf_counter()
                st = step()
                ctx.synchronize()
                ms = (time.perf_counter() - t0) * 1e3
                k = ctx.icp_kernel_ms()
                if r > 0:
                    out[v]["step"].append(ms)
                    out[v]["icp"].append(k)
                    out[v]["gn"].append((ms - k - ctx.kdtree_build_ms()) / st["iterations"])
            err.setdefault(st["final_error"], []).append(v)
    assert len(err) == 1, f"final errors differ: {err}"
for v in vals:
    o = {k: float(np.median(a)) for k, a in out[v].items()}
    print(f"{setting}={v}: ms/step {o['step']:.3f}  icp {o['icp']:.3f}  gn/iter {o['gn']:.4f}")
