#!/usr/bin/env python3
"""Where an ICP workgroup's life goes before its first iteration (lib/libdpg_setupclk.so): wave 0
of every workgroup stamps its set-up steps; this prints their medians / means per workgroup and
the set-up's share of the workgroup's life, for config 4 back to back.
usage: DPGSLAM_LIB=dpg-slam_amd/lib/libdpg_setupclk.so python tools/icp_setup_clock.py"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpg-slam_amd"))
from dpgslam import _abi, api, synth  # noqa: E402

w = synth.generate(os.environ.get("ICP_CONFIG", "config4"))
p = _abi.default_icp_params()
L = _abi.lib()
L.dpg_icp_setup_clock.argtypes = [C.POINTER(C.c_ulonglong), C.c_int64]
E = w.E
buf = (C.c_ulonglong * (E * 10))()
with api.Context(0) as ctx:
    ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
    ctx.icp_prepare(w.edges, w.est, p)
    for _ in range(4):
        ctx.icp_run(compute_cov=False)
        ctx.synchronize()
    kms = ctx.icp_kernel_ms()
    assert L.dpg_icp_setup_clock(buf, E) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(E, 10).astype(np.float64)
steps = np.diff(a[:, 0:8], axis=1)   # 7 steps
names = ["target recs", "source keys", "buckets", "barrier", "transform", "barrier", "iterations"]
life = a[:, 7] - a[:, 0]
ghz = (a[:, 7] - a[:, 0]) / ((a[:, 9] - a[:, 8]) * 10.0)
print(f"kernel {kms:.3f} ms, {E} workgroups; shader clock median {np.median(ghz):.3f} GHz")
print(f"workgroup life: median {np.median(life):.0f} ticks, mean {life.mean():.0f}")
for q, n in enumerate(names):
    print(f"  {n:12s} median {np.median(steps[:, q]):9.0f}  mean {steps[:, q].mean():9.0f}  share of life "
          f"{steps[:, q].sum() / life.sum():.1%}")
setup = a[:, 6] - a[:, 0]
print(f"set-up total: median {np.median(setup):.0f} ticks, mean {setup.mean():.0f}, {setup.sum() / life.sum():.1%} of "
      f"workgroup life")
# the first wave of workgroups (they start together) against the rest
t0 = a[:, 8]
first = t0 <= np.percentile(t0, 5)
print(f"first 5% to start: set-up mean {setup[first].mean():.0f}; the rest {setup[~first].mean():.0f}")
