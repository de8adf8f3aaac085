#!/usr/bin/env python3
"""What makes the ICP launch of the bench step slower than a back-to-back one?  The staged config-4
batch timed (HIP events) after each of: another ICP launch (+ host sync), the GN solve, a 1 GiB
memset (evicts L2 and the MALL, GPU busy), ~4 ms of compute-only work (a small matmul loop: busy,
caches kept), a 4 ms host sleep (idle).  Each condition runs in its own block of rounds so the
conditions do not leak into each other; the first launch of every block is dropped.
usage: python tools/icp_state_probe.py [rounds]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpg-slam_amd"))
from dpgslam import _abi, api, synth  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 12
w = synth.generate("config4")
p = _abi.default_icp_params()
gp = _abi.default_gn_params()
X0 = w.est.astype(np.float64)
dev = torch.device("cuda", 0)
big = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
a = torch.randn(256, 256, device=dev)
with api.Context(0) as ctx:
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
    ctx.icp_prepare(w.edges, w.est, p)
    ctx.gn_setup(w.V, w.factors_placeholder(), params=gp)
    ctx.icp_run(compute_cov=False)
    ctx.gn_take_icp(w.icp_factor_first, w.E, w.n_successive, p)
    ctx.synchronize()

    def gn():
        ctx.gn_set_poses(X0)
        ctx.gn_run()

    def busy():   # compute-only: ~4 ms of 256x256 matmuls on a few CUs' worth of data
        b = a
        for _ in range(400):
            b = torch.mm(b, a) * 1e-3

    t0 = time.perf_counter()
    busy(); torch.cuda.synchronize()
    busy_ms = (time.perf_counter() - t0) * 1e3
    pre = {"after-icp": lambda: ctx.icp_run(compute_cov=False), "after-gn": gn,
           "after-memset-1GiB": lambda: big.fill_(1), "after-busy-compute": busy,
           "after-idle-4ms": lambda: time.sleep(0.004), "none (sync gap only)": lambda: None,
           "after-gn+memset-1GiB": lambda: (gn(), big.fill_(2)),
           "after-gn+memset-64MiB": lambda: (gn(), big[:1 << 26].fill_(3)),
           "after-gn+memset-8MiB": lambda: (gn(), big[:1 << 23].fill_(4)),
           "after-idle+memset-64MiB": lambda: (time.sleep(0.004), big[:1 << 26].fill_(5)),
           "after-gn+read-1GiB": lambda: (gn(), big.sum(dtype=torch.int64)),
           "after-gn+busy-compute": lambda: (gn(), busy())}
    if len(sys.argv) > 2:
        pre = {k: v for k, v in pre.items() if "+" in k or k in ("after-gn", "after-icp")}
    for k, f in pre.items():
        ms = []
        for r in range(rounds + 1):
            f()   # no synchronisation: the ICP is queued behind it, as in the bench step
            ctx.icp_run(compute_cov=False)
            ctx.synchronize()
            torch.cuda.synchronize()
            if r > 0:
                ms.append(ctx.icp_kernel_ms())
        print(f"{k:22s} icp kernel median {np.median(ms):.3f} ms  min {np.min(ms):.3f}  max {np.max(ms):.3f}", flush=True)
    print(f"(busy block {busy_ms:.1f} ms)")
