#!/usr/bin/env python3
"""GN with factorization reuse (chord steps) on config4: iterations, factorizations, time and the
pose difference to plain Gauss-Newton, for several refactor thresholds (GPU)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpg-slam_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

torch.cuda.init()
from dpgslam import _abi, api, synth  # noqa: E402
from graphs import pose_diff  # noqa: E402

w = synth.generate(sys.argv[1] if len(sys.argv) > 1 else "config4")
p = _abi.default_icp_params()
with api.Context(0) as ctx:
    ctx.upload_scans(w.pts, w.offsets, 5)
    res, _ = ctx.icp_batch(w.edges, w.est, p, compute_cov=False)
    F = w.factors_with_icp(res, p)
    X0 = w.est.astype(np.float64)
    ref = None
    for reuse, tau in [(0, 0.0), (1, 1e-4), (1, 1e-3), (1, 1e-2), (1, 1e-1)]:
        gp = _abi.default_gn_params()
        gp.reuse_factorization, gp.refactor_delta = reuse, tau
        ctx.optimize_graph(X0, F, gp)   # warm
        t0 = time.perf_counter()
        X, st = ctx.optimize_graph(X0, F, gp)
        ms = (time.perf_counter() - t0) * 1e3
        nf = ctx.gn_factorizations()
        if ref is None:
            ref = X
        print(f"reuse={reuse} tau={tau:g}: iterations {st.iterations} factorizations {nf} {ms:.2f} ms "
              f"last|d| {st.last_delta_inf:.2e} max pose diff to GN {np.abs(pose_diff(X, ref)).max():.2e}", flush=True)
