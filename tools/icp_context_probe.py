#!/usr/bin/env python3
"""Why the ICP kernel times longer inside bench.py's step than in tools/icp_var_ab.py: the same
launch (config 4, one context) timed (a) back to back, (b) right after the step's GN loop, (c) after
the GN loop and a host sleep, (d) with the GN loop on but the covariance kernel off, (e) after GN
and another ICP, (f, g) after the GN loop and a 0.1 / 1 ms host sleep, (h) after an ICP and a 5 ms
sleep (idle without a GN before it), interleaved."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpg-slam_amd"))
from dpgslam import _abi, api, synth  # noqa: E402

rounds = int(os.environ.get("AB_ROUNDS", "7"))
w = synth.generate(os.environ.get("ICP_CONFIG", "config4"))
p = _abi.default_icp_params()
gp = _abi.default_gn_params()
ms = {k: [] for k in ("a_back_to_back", "b_after_gn", "c_after_gn_sleep5ms", "d_after_gn_nocov", "e_after_gn_cov_icp",
                      "f_after_gn_sleep0.1ms", "g_after_gn_sleep1ms", "h_icp_sleep5ms")}
with api.Context(0) as ctx:
    if os.environ.get("PROBE_TORCH_STREAM") == "1":   # bench.py's setting: torch's current stream
        import torch
        ctx.set_stream(torch.cuda.current_stream(torch.device("cuda", 0)).cuda_stream)
        print("on torch's current stream")
    ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
    ctx.icp_prepare(w.edges, w.est, p)
    F = w.factors_placeholder()
    ctx.gn_setup(w.V, F, (0, len(F)), gp)
    X0 = w.est.astype(np.float64)

    def gn():
        ctx.gn_take_icp(w.icp_factor_first, w.E, w.n_successive, p)
        ctx.gn_set_poses(X0)
        ctx.gn_run()

    for r in range(rounds + 1):
        for k in ms:
            if k == "a_back_to_back":
                ctx.icp_run(compute_cov=True)
            elif k == "b_after_gn":
                ctx.icp_run(compute_cov=True)
                gn()
            elif k == "c_after_gn_sleep5ms":
                ctx.icp_run(compute_cov=True)
                gn()
                ctx.synchronize()
                time.sleep(0.005)
            elif k in ("f_after_gn_sleep0.1ms", "g_after_gn_sleep1ms"):
                ctx.icp_run(compute_cov=True)
                gn()
                ctx.synchronize()
                time.sleep(0.0001 if k.startswith("f") else 0.001)
            elif k == "h_icp_sleep5ms":   # idle alone, no GN before it
                ctx.icp_run(compute_cov=True)
                ctx.synchronize()
                time.sleep(0.005)
            elif k == "d_after_gn_nocov":
                ctx.icp_run(compute_cov=False)
                ctx.gn_set_poses(X0)
                ctx.gn_run()
            else:
                ctx.icp_run(compute_cov=True)
                gn()
                ctx.icp_run(compute_cov=True)
            ctx.icp_run(compute_cov=True)
            ctx.synchronize()
            if r > 0:
                ms[k].append(ctx.icp_kernel_ms())
for k, v in ms.items():
    a = np.array(v)
    print(f"{k:24s} icp kernel median {np.median(a):.3f} ms  min {a.min():.3f}  max {a.max():.3f}")
