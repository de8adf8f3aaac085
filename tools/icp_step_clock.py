#!/usr/bin/env python3
"""The ICP kernel's per-phase clock in bench.py's step placement against back to back (VERDICT r5
next-1 step 1): with lib/libdpg_timing.so (DPGSLAM_LIB) the same config-4 launch is run
  step -- exactly bench.py's step (torch's current stream, ICP + covariance, gn_take_icp,
          gn_set_poses, gn_run, synchronize, the bench's per-step event reads);
  b2b  -- icp_run back to back, one synchronize per launch;
interleaved, STEPS launches each per round; the clock counters are read per placement (reset before
each placement's launches), so each phase's ticks per wave-iteration can be set side by side.  With
the plain lib (no counters) it reports the kernel times only.
usage: DPGSLAM_LIB=dpg-slam_amd/lib/libdpg_timing.so python tools/icp_step_clock.py"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpg-slam_amd"))
import torch  # noqa: E402
from dpgslam import _abi, api, synth  # noqa: E402

rounds = int(os.environ.get("AB_ROUNDS", "4"))
steps = int(os.environ.get("STEPS", "5"))
w = synth.generate(os.environ.get("ICP_CONFIG", "config4"))
p = _abi.default_icp_params()
gp = _abi.default_gn_params()
L = _abi.lib()
timing = hasattr(L, "dpg_icp_stats")
if timing:
    L.dpg_icp_stats.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
names = ["search", "sums+fold", "arrive+fit+barrier", "move+barrier", "queue (barriers, scans)"]
clock = {k: np.zeros(17) for k in ("step", "b2b")}
kms = {k: [] for k in ("step", "b2b")}
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
with api.Context(0) as ctx:
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
    ctx.icp_prepare(w.edges, w.est, p)
    F = w.factors_placeholder()
    ctx.gn_setup(w.V, F, params=gp)
    X0 = w.est.astype(np.float64)

    def step():
        ctx.icp_run(compute_cov=True)
        ctx.gn_take_icp(w.icp_factor_first, w.E, w.n_successive, p)
        ctx.gn_set_poses(X0)
        ctx.gn_run()
        ctx.synchronize()
        k = ctx.icp_kernel_ms()
        ctx.cov_kernel_ms()
        ctx.kdtree_build_ms()
        ctx.gn_factorizations()
        return k

    def b2b():
        ctx.icp_run(compute_cov=False)
        ctx.synchronize()
        return ctx.icp_kernel_ms()

    st = (C.c_ulonglong * 64)()
    for _ in range(3):   # warm-up: the measured schedule is learnt from the first run
        step()
    for r in range(rounds):
        for name, fn in (("step", step), ("b2b", b2b)):
            fn()   # the placement's own lead-in (not counted)
            if timing:
                L.dpg_icp_stats(st, 1)
            for _ in range(steps):
                kms[name].append(fn())
            if timing:
                L.dpg_icp_stats(st, 0)
                s = list(st)
                clock[name] += np.array(s[8:12] + [s[45], s[12], s[40], s[41], s[42], s[43], s[47]] + s[48:54],
                                        dtype=np.float64)
for name in ("step", "b2b"):
    a = np.array(kms[name])
    print(f"{name:5s} icp kernel median {np.median(a):.3f} ms  min {a.min():.3f}  max {a.max():.3f}  ({len(a)} launches)")
if timing:
    print("per wave-iteration clock (s_memtime ticks):  step   b2b   diff")
    for q, n in enumerate(names):
        a, b = clock["step"][q] / clock["step"][5], clock["b2b"][q] / clock["b2b"][5]
        print(f"  {n:24s} {a:8.0f} {b:8.0f} {a - b:+7.0f}")
    a = clock["step"][:5].sum() / clock["step"][5]
    b = clock["b2b"][:5].sum() / clock["b2b"][5]
    print(f"  {'total':24s} {a:8.0f} {b:8.0f} {a - b:+7.0f}")
    for name in ("step", "b2b"):
        c = clock[name]
        print(f"{name:5s} per wave: set-up {c[6] / c[9]:.0f} shader ticks, whole {c[7] / c[9]:.0f} shader ticks over "
              f"{c[8] / c[9] * 10:.0f} ns -> shader clock {c[7] / c[8] * 0.1:.3f} GHz")
        print("      set-up steps (shader ticks per wave): " + "  ".join(
            f"{n} {v / c[9]:.0f}" for n, v in zip(["entry->edge", "target recs", "source keys", "buckets", "barrier",
                                                  "transform", "barrier"], c[10:17])))
