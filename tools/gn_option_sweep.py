#!/usr/bin/env python3
"""GN-only sweep of the Cholesky's solver options on config 4's graph (one ICP run for the
factors, then per option set: gn_setup, then gn_run from the same poses, interleaved rounds; the
final error must match the first set's).  usage: python tools/gn_option_sweep.py
'solve_stage=-1' 'solve_stage=4096' ...  (fields of dpg_solver_options, comma separated)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpg-slam_amd"))
from dpgslam import _abi, api, synth  # noqa: E402

sets = sys.argv[1:] or ["solve_stage=-1"]
rounds = int(os.environ.get("AB_ROUNDS", "5"))
w = synth.generate(os.environ.get("GN_CONFIG", "config4"))
p = _abi.default_icp_params()
gp = _abi.default_gn_params()
X0 = w.est.astype(np.float64)
ms = {s: [] for s in sets}
with api.Context(0) as c:
    c.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
    c.icp_prepare(w.edges, w.est, p)
    c.icp_run(compute_cov=False)
    c.synchronize()
    F = w.factors_placeholder()
    ref = None
    for r in range(rounds + 1):
        for s in sets:
            kw = {}
            for kv in s.split(","):
                k, v = kv.split("=")
                kw[k] = float(v) if k == "relax_fraction" else int(v)
            c.set_solver_options(**kw)
            c.gn_setup(w.V, F, params=gp)
            c.gn_take_icp(w.icp_factor_first, w.E, w.n_successive, p)
            c.gn_set_poses(X0)
            st, _ = c.gn_run()
            c.synchronize()
            key = (st["iterations"], st["final_error"])
            if ref is None:
                ref = key
            if key != ref:
                print(f"{s}: DIFFERENT result {key} vs {ref}")
            if r > 0:
                ms[s].append(st["ms_per_iteration"])
for s in sets:
    print(f"{s:40s} ms/iter median {np.median(ms[s]):.4f} min {np.min(ms[s]):.4f}")
print("reference", ref)
