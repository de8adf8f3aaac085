"""Dump the incremental bench's graph arrival sequence (bench.py --workload incremental: node v
brings the pair (v-1, v) and the config's loop closures (j, v)) for tools/incsym_bench.cpp.

usage: python tools/dump_inc_edges.py [config4] [V] [out.bin]
format: int32 V, then per node: int32 count, count x (int32 lo, int32 hi)
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dpg-slam_amd"))
from dpgslam import synth  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "config4"
    V = int(sys.argv[2]) if len(sys.argv) > 2 else 5000
    out = sys.argv[3] if len(sys.argv) > 3 else "/tmp/inc_edges.bin"
    w = synth.generate(cfg)
    V = min(V, w.V)
    by_node = [[] for _ in range(V)]
    for v in range(1, V):
        by_node[v].append((v - 1, v))
    for j, i in w.edges[w.n_successive:]:
        if i < V and (int(j), int(i)) != (int(i) - 1, int(i)):
            by_node[int(i)].append((int(min(i, j)), int(max(i, j))))
    buf = [np.int32(V)]
    for b in by_node:
        buf.append(np.int32(len(b)))
        buf.extend(np.int32(x) for e in b for x in e)
    np.asarray(buf, np.int32).tofile(out)
    print(f"{cfg}: V={V}, pairs={sum(len(b) for b in by_node)} -> {out}")


if __name__ == "__main__":
    main()
