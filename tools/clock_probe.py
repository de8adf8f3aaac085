#!/usr/bin/env python3
"""Diagnostics: the shader clock over time after different preceding activity (tools/clk/
clock_probe.hip: s_memtime / s_memrealtime per 50 us window, a full-chip VALU load), and the GN
solve's time with and without a concurrent VALU load on a second stream.
usage: python tools/clock_probe.py"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpg-slam_amd"))
from dpgslam import _abi, api, synth  # noqa: E402

lib = ctypes.CDLL(os.path.join(ROOT, "tools", "clk", "libclock_probe.so"))
dev = torch.device("cuda", 0)
s_main = torch.cuda.current_stream(dev)
s_side = torch.cuda.Stream(dev, priority=0)
NW = 60
out = torch.zeros(2 * NW, dtype=torch.int64, device=dev)
sink = torch.zeros(1024, dtype=torch.float32, device=dev)
big = torch.empty(1 << 30, dtype=torch.uint8, device=dev)


def trace(label):
    lib.clk_trace_launch(ctypes.c_void_p(out.data_ptr()), 1024, 256, NW, 5000, ctypes.c_void_p(s_main.cuda_stream))
    torch.cuda.synchronize()
    o = out.cpu().numpy().reshape(NW, 2)
    mhz = o[:, 0] / o[:, 1] * 100.0
    print(f"{label:18s} MHz per 50us window: " + " ".join(f"{m:.0f}" for m in mhz[:12]) + " ... " +
          " ".join(f"{m:.0f}" for m in mhz[-4:]) + f"   (mean first 1 ms {mhz[:20].mean():.0f}, last 1 ms {mhz[-20:].mean():.0f})",
          flush=True)


w = synth.generate("config4")
p = _abi.default_icp_params()
gp = _abi.default_gn_params()
X0 = w.est.astype(np.float64)
with api.Context(0) as ctx:
    ctx.set_stream(s_main.cuda_stream)
    ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
    ctx.icp_prepare(w.edges, w.est, p)
    ctx.gn_setup(w.V, w.factors_placeholder(), params=gp)
    ctx.icp_run(compute_cov=False)
    ctx.gn_take_icp(w.icp_factor_first, w.E, w.n_successive, p)
    ctx.synchronize()

    def gn():
        ctx.gn_set_poses(X0)
        ctx.gn_run()

    for rep in range(2):
        time.sleep(0.004); trace("after-idle-4ms")
        time.sleep(0.05); trace("after-idle-50ms")
        big.fill_(1); trace("after-memset")
        gn(); trace("after-gn")
        ctx.icp_run(compute_cov=False); trace("after-icp")
        trace("after-clk-trace")

    # GN with / without a concurrent VALU load on the side stream
    def heat(iters, blocks):
        with torch.cuda.stream(s_side):
            lib.heat_launch(blocks, 256, iters, ctypes.c_void_p(sink.data_ptr()), ctypes.c_void_p(s_side.cuda_stream))

    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s_side):
        e0.record(s_side); heat(20000, 128); e1.record(s_side)
    torch.cuda.synchronize()
    per = e0.elapsed_time(e1) / 20000
    iters = int(6.0 / per)
    print(f"heater: {per * 1e3:.3f} us per 1000 iterations at 128 blocks -> {iters} iterations ~ 6 ms", flush=True)
    for blocks in (0, 64, 256):
        ts = []
        for r in range(8):
            ctx.icp_run(compute_cov=False)
            ctx.synchronize(); torch.cuda.synchronize()
            if blocks:
                heat(iters, blocks)
            t0 = time.perf_counter()
            gn()
            ctx.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
            torch.cuda.synchronize()
        print(f"GN solve with heater blocks={blocks:4d}: median {np.median(ts[2:]):.3f} ms  min {min(ts[2:]):.3f}", flush=True)
    # the bench step's ICP after a GN that ran beside the heater
    for blocks in (0, 64):
        ms = []
        for r in range(8):
            if blocks:
                heat(iters, blocks)
            gn()
            ctx.icp_run(compute_cov=False)
            ctx.synchronize(); torch.cuda.synchronize()
            ms.append(ctx.icp_kernel_ms())
        print(f"ICP after GN, heater blocks={blocks:3d}: median {np.median(ms[2:]):.3f} ms", flush=True)
