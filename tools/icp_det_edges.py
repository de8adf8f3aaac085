#!/usr/bin/env python3
"""Determinism of one angular ICP kernel variant on a few chosen edges, run many times with the
per-iteration correspondence trace: every run against the oracle (brute-force nn), and for a run
that differs, the first iteration / points where its trace leaves a good run's.
usage: python tools/icp_det_edges.py VARIANT CONFIG RUNS EDGE...  (SWEEP=1: offset = run)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpg-slam_amd"))
sys.path.insert(0, ROOT)
from dpgslam import _abi, api, synth  # noqa: E402
from oracle import oracle  # noqa: E402

v, cfg, runs = int(sys.argv[1]), sys.argv[2], int(sys.argv[3])
sel = [int(a) for a in sys.argv[4:]]
w = synth.generate(cfg)
p = _abi.default_icp_params()
want, _ = oracle.icp_batch(w.pts, w.offsets, w.edges[sel], w.est, p, nn=oracle.NN_BRUTE)
rep = int(os.environ.get("REP", "1"))   # the edges repeated REP times in one batch (a full chip)
E = np.tile(w.edges[sel], (rep, 1))
want = np.tile(want, rep)
TI = int(os.environ.get("TI", "60"))
good = {}
nbad = 0
with api.Context(0) as ctx:
    ctx.set_icp_schedule("caller")
    ctx.set_icp_kernel_variant(v)
    ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
    bad_runs = []
    for r in range(runs):
        if os.environ.get("SWEEP"):   # variant 5: a different affine permutation per run
            ctx.set_icp_kernel_variant(v + 256 * r)
        res, _ = ctx.icp_batch(E, w.est, p, compute_cov=False, trace_iters=TI)
        tr = ctx.icp_fetch_trace(TI)
        for j in range(len(E)):
            ok = res[j].tobytes() == want[j].tobytes()
            if ok and j % len(sel) not in good:
                good[j % len(sel)] = tr[j].copy()
            if not ok:
                nbad += 1
                bad_runs.append((r, j, res[j].copy(), tr[j].copy()))
    print(f"variant {v}: {nbad} wrong results in {runs} runs x {len(E)} edges")
    for r, j, rj, tj in bad_runs[:6]:
        print(f"run {r} edge {sel[j % len(sel)]} (copy {j // len(sel)}): {rj}\n   oracle {want[j]}")
        g = good.get(j % len(sel))
        if g is not None:
            d = np.nonzero((tj != g).any(1))[0]
            if len(d):
                k = d[0]
                pts = np.nonzero(tj[k] != g[k])[0]
                print(f"   trace differs first at iteration {k}: points {pts[:8]} bad {tj[k, pts[:8]]} good {g[k, pts[:8]]}")
            else:
                print("   trace identical to a good run's: the sums, not the search")
        else:
            print("   no good run of this edge to compare")
