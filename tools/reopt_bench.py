#!/usr/bin/env python3
"""Re-linearisation sweep (DpgSLAM::reoptimize, dpg_slam.cc:35-120) timed on the GPU: config 2's
500 nodes split into two passes -- every loop-closure candidate of the reference's distance rule
(5 m within a pass, 2 m across) aligned in one batch, then the batch GN.  Prints one JSON line with
the phase times and the sweep's ICP edges/s; the oracle (1 thread) aligns a bounded sample of the
same edges for the CPU baseline.
usage: PYTHONPATH=.:dpg-slam_amd python tools/reopt_bench.py [config] [reps]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpg-slam_amd")]
from dpgslam import api, synth  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "config2"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
w = synth.generate(name)
passes = np.zeros(w.V, np.int32)
passes[w.V // 2:] = 1
out = {"workload": f"{name}: {w.V} nodes, 2 passes, reoptimize sweep"}
with api.Context(0) as ctx:
    ctx.upload_scans(w.pts, w.offsets, 5)
    X, st = ctx.reoptimize(passes, w.est, w.odom)   # warm-up (symbolic analysis, allocations)
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        X, st = ctx.reoptimize(passes, w.est, w.odom)
        t.append(time.perf_counter() - t0)
    ms = 1e3 * float(np.median(t))
    out.update({"ms_sweep": ms, "icp_edges": int(st.n_icp_edges), "candidates": int(st.n_candidates),
                "loop_closures": int(st.n_loop_closures), "factors": int(st.n_factors),
                "ms_candidates": st.ms_candidates, "ms_icp": st.ms_icp, "ms_gn": st.ms_gn,
                "gn_iterations": st.gn.iterations, "sweep_icp_edges_per_s": st.n_icp_edges / (st.ms_icp * 1e-3)})
    edges = np.concatenate([np.stack([np.arange(w.V - 1), np.arange(1, w.V)], 1),
                            ctx.loop_closure_candidates(w.est, passes)]).astype(np.int32)
from oracle import oracle as O  # noqa: E402
rng = np.random.default_rng(0)
sel = np.sort(rng.choice(len(edges), min(400, len(edges)), replace=False))
t0 = time.perf_counter()
O.icp_batch(w.pts, w.offsets, edges[sel], w.est, None, O.NN_GRID, 1)
dt = time.perf_counter() - t0
out["cpu_baseline"] = {"value": len(sel) / dt, "unit": "edges/s", "cores": 1, "kind": "port",
                       "sample": f"oracle ICP on {len(sel)} random edges of the sweep ({dt:.1f} s)"}
print(json.dumps(out))
