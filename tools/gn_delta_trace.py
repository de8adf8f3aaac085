#!/usr/bin/env python3
"""The Gauss-Newton trajectory of config 4's step under several chord thresholds (refactor_delta):
max |delta| after each iteration (dpg_optimize_graph truncated at m = 1, 2, ... iterations from the
same start), and the largest pose difference of the converged solve to the oracle's plain GN.
usage: python tools/gn_delta_trace.py [deltas...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpg-slam_amd"), os.path.join(ROOT, "tests")]
from dpgslam import _abi, api, synth  # noqa: E402
from oracle import oracle as O  # noqa: E402
from conftest import angle_wrap  # noqa: E402

deltas = [float(x) for x in sys.argv[1:]] or [1e-3, 1e-2, 0.1]
w = synth.generate("config4")
p = _abi.default_icp_params()
with api.Context(0) as ctx:
    ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
    res, _ = ctx.icp_batch(w.edges, w.est, p, compute_cov=False)
    F = w.factors_with_icp(res, p)
    X0 = w.est.astype(np.float64)
    Xo, sto = O.optimize_graph(X0, F)
    print(f"oracle plain GN: {sto.iterations} iterations, final error {sto.final_error:.12e}", flush=True)
    for d in deltas:
        gp = _abi.default_gn_params()
        gp.refactor_delta = d
        traj = []
        for m in range(1, 16):
            gp.max_iterations = m
            X, st = ctx.optimize_graph(X0, F, gp)
            traj.append(st.last_delta_inf)
            if st.iterations < m:
                break
        gp.max_iterations = _abi.default_gn_params().max_iterations
        X, st = ctx.optimize_graph(X0, F, gp)
        dX = np.concatenate([X[:, :2] - Xo[:, :2], angle_wrap(X[:, 2:] - Xo[:, 2:])], 1)
        print(f"refactor_delta {d:g}: iterations {st.iterations}, max|delta| per iteration "
              + " ".join(f"{t:.2e}" for t in traj)
              + f" | final error {st.final_error:.12e}, max pose diff vs oracle {np.abs(dX).max():.2e}", flush=True)
