#!/usr/bin/env python3
"""Does a fresh context's first batched ICP run beside the host's GN setup?  Times each call of
bench.py's cold single solve separately (config from argv, default config4)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpg-slam_amd"))
from dpgslam import _abi, api, synth  # noqa: E402

w = synth.generate(sys.argv[1] if len(sys.argv) > 1 else "config4")
p = _abi.default_icp_params()
gp = _abi.default_gn_params()
for rep in range(3):
    with api.Context(0) as c:
        c.synchronize()
        t = [time.perf_counter()]
        c.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
        t.append(time.perf_counter())
        c.icp_prepare(w.edges, w.est, p)
        c.synchronize()
        t.append(time.perf_counter())
        c.icp_run(compute_cov=True)
        t.append(time.perf_counter())
        F = w.factors_placeholder()
        c.gn_setup(w.V, F, params=gp)
        t.append(time.perf_counter())
        c.synchronize()
        t.append(time.perf_counter())
        d = np.diff(t) * 1e3
        print(f"upload {d[0]:.2f}  prepare {d[1]:.2f}  icp_run call {d[2]:.2f}  gn_setup call {d[3]:.2f}  sync {d[4]:.2f}  "
              f"| icp kernel {c.icp_kernel_ms():.2f} index {c.kdtree_build_ms():.3f} cov {c.cov_kernel_ms():.2f} "
              f"| setup parts {c.gn_setup_profile()}", flush=True)
