#!/usr/bin/env python3
"""ICP diagnostics on config4 (GPU): candidate counters with the lib/libdpg_stats.so build,
per-phase clock with the lib/libdpg_timing.so build:
   DPGSLAM_LIB=dpg-slam_amd/lib/libdpg_stats.so python tools/icp_stats.py
   DPGSLAM_LIB=dpg-slam_amd/lib/libdpg_timing.so python tools/icp_stats.py"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpg-slam_amd"))
from dpgslam import _abi, api, synth  # noqa: E402

import argparse  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("config", nargs="?", default="config4")
ap.add_argument("--cap", action="store_true", help="transformation epsilon 0 and MSE threshold 0: every edge runs "
                                                   "to the iteration cap")
ap.add_argument("--edges", type=int, default=0, help="only the first N edges")
ap.add_argument("--variant", type=int, default=0, help="angular kernel form (dpg_ctx_set_icp_kernel_variant)")
a = ap.parse_args()
w = synth.generate(a.config)
p = _abi.default_icp_params()
if a.cap:
    p.icp_maximum_transformation_epsilon = 0.0
    p.mse_threshold_absolute = 0.0
if a.edges:
    w.edges = w.edges[:a.edges]
L = _abi.lib()
L.dpg_icp_stats.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
st = (C.c_ulonglong * 64)()
with api.Context(0) as ctx:
    if os.environ.get("DPG_DEFER_CAP"):
        ctx.set_icp_defer_cap(int(os.environ["DPG_DEFER_CAP"]))
    ctx.set_icp_kernel_variant(a.variant)
    ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
    ctx.icp_prepare(w.edges, w.est, p)
    L.dpg_icp_stats(st, 1)
    ctx.icp_run(compute_cov=False)
    ctx.synchronize()
    L.dpg_icp_stats(st, 0)
    res, _ = ctx.icp_fetch(with_hessian=False)
it = res["iterations"]
s = list(st)
print(f"edges {len(it)}  iterations mean {it.mean():.2f} p50 {np.median(it):.0f} p99 {np.percentile(it, 99):.0f} max {it.max()}"
      f"  sum {it.sum()}")
if s[0]:
  print(f"point-iterations {s[0]}  correspondences {s[5]} ({s[5] / s[0]:.2%})  no fwd match {s[6]} ({s[6] / s[0]:.2%})"
      f"  full-scan windows {s[7]}")
  KU = 4   # candidates per wave trip (dpg_icp_ang.hip kU)
  print(f"forward: candidates/point {s[1] / s[0]:.1f}  wave-level candidates/point-slot {KU * s[2] * 64 / s[0]:.1f}")
  print(f"full-scan reciprocal windows {s[13]}  wave imbalance (slowest wave trips x 8 / all trips) {8 * s[14] / max(1, s[15]):.2f}")
  print(f"reciprocal: candidates/matched {s[3] / max(1, s[5]):.1f}  wave-level candidates/point-slot {KU * s[4] * 64 / s[0]:.1f}")
if s[0]:
  print(f"queue: forward items {s[40]} (candidates/item {s[41] / max(1, s[40]):.0f}), cooperative reciprocal scans {s[42]}"
        f" (candidates/scan {s[43] / max(1, s[42]):.0f}), workgroup-iterations with a queue {s[44]}")
if s[0]:
  bins = ["0", "1", "2", "3", "4", "5-8", "9-16", "17-32", "33-64", "65-128", "129-256", ">256"]
  for name, o in (("forward", 16), ("reciprocal", 28)):
    t = sum(s[o:o + 12])
    print(f"{name} wave trips by trips-per-slot bin (share of all {name} trips): " +
          " ".join(f"{b}:{s[o + k] / max(1, t):.1%}" for k, b in enumerate(bins)))
if s[0]:
  import struct
  f = lambda u: struct.unpack("<f", struct.pack("<I", u & 0xffffffff))[0]   # noqa: E731
  print(f"drift: max |moved - F p| {f(s[46]):.3e} m, max drift / window margin {f(s[47]):.4f}")
tot = sum(s[8:12]) + s[45]
if s[12]:
    names = ["search", "sums+fold", "arrive+fit+barrier", "move+barrier", "queue (barriers, scans)"]
    print(f"per wave-iteration clock (s_memtime ticks, {s[12]} wave-iterations):")
    for n, v in zip(names, s[8:12] + [s[45]]):
        print(f"  {n:22s} {v / s[12]:9.0f}  ({v / tot:.1%})")
