#!/usr/bin/env python3
"""The ICP shard tail at N = 2, 4, 8 on one card: a context of N virtual devices
(dpg_ctx_create_virtual) runs each device's share as its own kernel, one after the other on the
shared stream, so dpg_icp_batch_kernel_ms (the slowest device) is the slowest share's solo
duration -- what that rank takes on its own GPU.  Both dispatch schedules: "caller" (e mod N,
caller order) and "measured" (LPT over the last run's iterations x points, longest first).  The
tail is then set against 1/N of the single-device launch and against the longest single
alignment run alone (the floor no assignment can go below).
usage: python tools/icp_lpt_probe.py [config] [reps] [kernel variant]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpg-slam_amd"))
from dpgslam import _abi, api, synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "config4"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
kvar = int(sys.argv[3]) if len(sys.argv) > 3 else 0   # angular kernel form (6 / 7: two / three workgroups per CU)
w = synth.generate(cfg)
p = _abi.default_icp_params()


def timed(ctx, n):
    ms = []
    for _ in range(n):
        ctx.icp_run(compute_cov=False)
        ms.append(ctx.icp_kernel_ms())
    return float(np.median(ms)), float(np.min(ms))


with api.Context(0) as c1:
    c1.set_icp_schedule("measured")
    c1.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
    c1.icp_prepare(w.edges, w.est, p)
    c1.icp_run(compute_cov=False)
    full, _ = timed(c1, reps)
    res, _ = c1.icp_fetch(with_hessian=False)
    it = res["iterations"]
    longest = int(np.argmax(it * np.diff(w.offsets)[w.edges[:, 1]]))
    c1.icp_prepare(w.edges[longest:longest + 1], w.est, p)
    solo, _ = timed(c1, reps)
print(f"{cfg}: single device {full:.3f} ms for {w.E} edges; longest alignment alone (edge {longest}, "
      f"{it[longest]} iterations) {solo:.3f} ms")
for n in (2, 4, 8):
    row = []
    for sched in ("caller", "measured"):
        with api.Context(0, virtual=n) as c:
            c.set_icp_kernel_variant(kvar)
            c.set_icp_schedule(sched)
            c.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
            c.icp_prepare(w.edges, w.est, p)
            c.icp_run(compute_cov=False)   # measured: learns the costs (planned e mod N the first time)
            med, mn = timed(c, reps)
            r, _ = c.icp_fetch(with_hessian=False)
            assert r.tobytes() == res.tobytes(), "results differ from the single device"
            row.append(f"{sched} slowest share {med:.3f} ms (min {mn:.3f})")
    print(f"N={n}: 1/N of single {full / n:.3f} ms; " + "; ".join(row), flush=True)
