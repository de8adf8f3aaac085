#!/usr/bin/env python3
"""Per-node kernel timeline of the incremental bench from a rocprofv3 kernel trace (csv): mean
duration per kernel over the last 500 nodes and one typical node's launches (usage: trace.csv)."""
import collections
import csv
import sys

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
K = []
for r in rows:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    K.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n.split("(")[0][:40]))
K.sort()
starts = [i for i, k in enumerate(K) if k[2].startswith("icp_ang_kernel")]
nodes = [K[a:b] for a, b in zip(starts[:-1], starts[1:])]
tail = nodes[-520:-20]
dur = collections.defaultdict(list)
span = []
for nd in tail:
    for s, e, n in nd:
        dur[n].append((e - s) / 1e3)
    bw = [e for s, e, n in nd if n.startswith("chol_backward")]
    if bw:
        span.append((max(bw) - nd[0][0]) / 1e3)
for n, v in sorted(dur.items(), key=lambda x: -sum(x[1])):
    print(f"{n:42s} per node {len(v) / len(tail):5.2f} x mean {np.mean(v):8.1f} us = {sum(v) / len(tail):8.1f} us")
print("ICP kernel start -> backward end per node: median %.1f us" % np.median(span))
nd = tail[len(tail) // 2]
t0 = nd[0][0]
for s, e, n in nd:
    print(f"  {(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f}  {n}")
