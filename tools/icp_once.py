#!/usr/bin/env python3
"""Run the batched ICP of config 4 a few times (no covariance, no GN): the program the ICP kernel's
PMC passes profile (tools/icp_pmc_job.sh).  usage: python tools/icp_once.py [runs]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpg-slam_amd"))
from dpgslam import _abi, api, synth  # noqa: E402

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 2
w = synth.generate(os.environ.get("ICP_CONFIG", "config4"))
p = _abi.default_icp_params()
with api.Context(0) as ctx:
    ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
    ctx.icp_prepare(w.edges, w.est, p)
    for _ in range(runs):
        ctx.icp_run(compute_cov=False)
        ctx.synchronize()
        print(f"icp kernel {ctx.icp_kernel_ms():.3f} ms", flush=True)
