"""Debug helper: run the first executeDPG calls of the small dynamic workload on both paths and print
every counter side by side (GPU box)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "dpg-slam_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
from dpgslam import synth, api
from oracle import oracle as O

w = synth.make_dynamic(n_passes=3, nodes_per_pass=20, n_beams=360, world_size=20.0, range_max=8.0, n_boxes=10)
o = O.OracleDpgStore(w.ranges, w.geom)
ctx = api.Context(0)
g = api.DpgStore(ctx, w.ranges, w.geom)
for v in range(20, 24):
    cur = int(v - w.pass_start[w.pass_of[v]] + 1)
    so = o.execute_dpg(v + 1, cur, w.est[:v + 1]).counters()
    sg = g.execute_dpg(v + 1, cur, w.est[:v + 1]).counters()
    print(v, {k: (sg[k], so[k]) for k in so if sg[k] != so[k]}, so)
    lo, _, _ = o.fetch()
    lg, _, _ = g.fetch()
    d = np.nonzero(lo != lg)[0]
    print("  label diffs", len(d), [(int(i) // 360, int(i) % 360, int(lo[i]), int(lg[i])) for i in d[:12]])
    o.load(labels=lg, sector_active=g.fetch()[1], node_active=g.fetch()[2])
