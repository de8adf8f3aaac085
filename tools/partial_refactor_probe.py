#!/usr/bin/env python3
"""Partial vs full refactorization in lockstep on bench.py's incremental workload (config 4 node by
node through dpg_add_node_pairs): two contexts, one graph each (full_refactor 0 / 1); stops at the
first update whose estimate, error or status differs and prints that update's record."""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpg-slam_amd"))
from dpgslam import _abi, api, synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "config4"
V = int(sys.argv[2]) if len(sys.argv) > 2 else 5000
w = synth.generate(cfg)
V = min(V, w.V)
p = _abi.default_icp_params()
lc = w.edges[w.n_successive:]
by_node = [[] for _ in range(V)]
for j, i in lc:
    if i < V:
        by_node[int(i)].append((int(j), int(i)))
L = _abi.lib()
pbuf = (C.c_double * 12)()
t0 = time.time()
with api.Context(0) as ca, api.Context(0) as cb:
    gp = api.IncGraph(ca)
    gf = api.IncGraph(cb, full_refactor=True)
    kept = 0
    for v in range(V):
        pr = np.asarray(by_node[v], np.int32).reshape(-1, 2)
        res = []
        for g in (gp, gf):
            try:
                st = g.add_node_pairs(w.cloud(v), w.est[v], pr, extra=w.base_factors[v:v + 1], successive=v >= 1,
                                      icp_params=p)
                L.dpg_inc_last_profile(C.c_void_p(g.handle), pbuf, 12)
                res.append((st, list(pbuf)))
            except _abi.DpgError as e:
                res.append((e, list(pbuf)))
        (sp, pp), (sf, pf) = res
        bad = isinstance(sp, Exception) or isinstance(sf, Exception)
        if not bad:
            u, q = sp.update, sf.update
            kept += u.fronts_kept > 0
            bad = (u.error, u.last_delta_inf, u.relinearized, u.reordered) != (q.error, q.last_delta_inf, q.relinearized,
                                                                                q.reordered)
            if not bad and (v % 50 == 0 or v == V - 1):
                bad = not np.array_equal(gp.poses(), gf.poses())
        if bad:
            print(f"DIVERGED at node {v}: partial {sp!r} full {sf!r}")
            for name, s in (("partial", sp), ("full", sf)):
                if not isinstance(s, Exception):
                    u = s.update
                    print(f"  {name}: reordered {u.reordered} relin {u.relinearized} kept {u.fronts_kept} "
                          f"err {u.error!r} delta {u.last_delta_inf!r} nnz {u.nnz_l}")
            print("  partial profile", [round(x, 4) for x in pp])
            print("  full profile", [round(x, 4) for x in pf])
            print("  by_node", by_node[v])
            sys.exit(1)
        if v % 250 == 0:
            print(f"node {v}: identical; updates keeping fronts {kept}; {time.time() - t0:.0f}s", flush=True)
    print(f"all {V} updates identical; {kept} kept fronts", flush=True)
