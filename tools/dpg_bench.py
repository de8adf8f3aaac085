"""Config 5 (BASELINE.json configs[4]): DPG change detection on a 10k-node, 4-pass dynamic workload.

The node store holds all 10 000 scans (5000 beams, 30 m) on the GPU; the timed region runs
executeDPG (dpg_execute_dpg) after every node of the later passes in order, the way the reference
runs it after each node addition (dpg_slam.cc:125-140), with --stride selecting a subset of those
calls.  Prints one JSON line: calls/s, ms per call, ray samples per second, the raster kernels'
share, and the oracle (CPU restatement, 1 thread) timed on the first --cpu-calls calls of the same
sequence as the CPU baseline.  Run on the GPU box:
    python tools/dpg_bench.py [--passes 4 --nodes-per-pass 2500 --stride 1 --max-calls 2000]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpg-slam_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from dpgslam import api, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--passes", type=int, default=4)
    ap.add_argument("--nodes-per-pass", type=int, default=2500)
    ap.add_argument("--beams", type=int, default=5000)
    ap.add_argument("--stride", type=int, default=1)
    ap.add_argument("--max-calls", type=int, default=100000)
    ap.add_argument("--cpu-calls", type=int, default=3)
    ap.add_argument("--check-calls", type=int, default=0, help="compare the first N calls with the oracle")
    a = ap.parse_args()

    t = time.time()
    w = synth.make_dynamic(n_passes=a.passes, nodes_per_pass=a.nodes_per_pass, n_beams=a.beams)
    gen_s = time.time() - t
    ctx = api.Context(0)
    g = api.DpgStore(ctx, w.ranges, w.geom)
    calls = [v for v in range(int(w.pass_start[1]), w.V, a.stride)][:a.max_calls]

    def args(v):
        p = w.pass_of[v]
        return v + 1, int(v - w.pass_start[p] + 1), w.est[:v + 1]

    # warm-up on a throw-away store (same workload), then the timed sequence on a fresh one
    for v in calls[:3]:
        g.execute_dpg(*args(v))
    g.close()
    g = api.DpgStore(ctx, w.ranges, w.geom)
    ctx.synchronize()
    tot = {k: 0 for k in ("n_candidates", "n_submap_nodes", "n_added", "n_removed", "n_committed",
                          "n_sectors_deactivated", "n_nodes_deactivated")}
    samples = 0
    kern_ms = 0.0
    t0 = time.perf_counter()
    for v in calls:
        st = g.execute_dpg(*args(v))
        samples += st.n_samples
        kern_ms += st.ms_kernels
        for k in tot:
            tot[k] += getattr(st, k)
    wall = time.perf_counter() - t0
    n = len(calls)

    check = None
    if a.check_calls:
        from oracle import oracle as O
        o = O.OracleDpgStore(w.ranges, w.geom)
        g2 = api.DpgStore(ctx, w.ranges, w.geom)
        ok = True
        for v in calls[:a.check_calls]:
            so, sg = o.execute_dpg(*args(v)).counters(), g2.execute_dpg(*args(v)).counters()
            ok &= so == sg
        lo, so_, ao = o.fetch()
        lg, sg_, ag = g2.fetch()
        ok &= bool(np.array_equal(lo, lg) and np.array_equal(so_, sg_) and np.array_equal(ao, ag))
        check = {"calls": a.check_calls, "bit_exact": bool(ok)}

    cpu = None
    if a.cpu_calls:
        from oracle import oracle as O
        o = O.OracleDpgStore(w.ranges, w.geom)
        t1 = time.perf_counter()
        for v in calls[:a.cpu_calls]:
            o.execute_dpg(*args(v))
        cs = time.perf_counter() - t1
        cpu = {"value": a.cpu_calls / cs, "unit": "executeDPG calls/s", "cores": 1, "kind": "port",
               "sample": f"oracle (C++ restatement, hash-map grids, 1 thread): the first {a.cpu_calls} calls of the "
                         f"same sequence ({cs:.1f} s)"}

    print(json.dumps({
        "metric": "executeDPG calls/s on the config-5 dynamic workload (DPG change detection)",
        "value": n / wall, "unit": "calls/s", "higher_is_better": True,
        "ms_per_call": 1e3 * wall / n, "kernel_ms_per_call": kern_ms / n, "calls": n,
        "ray_samples_per_s": samples / wall, "samples_per_call": samples / n,
        "config": {"workload": f"config5: {a.passes} passes x {a.nodes_per_pass} nodes, {a.beams}-beam scans "
                               f"(30 m), 24 movable boxes, executeDPG after every node of passes 1..{a.passes - 1}"
                               + (f" (stride {a.stride})" if a.stride > 1 else ""),
                   "nodes": int(w.V), "beams": a.beams},
        "totals": tot, "generation_s": gen_s, "check": check, "cpu_baseline": cpu,
        "data": "synthetic (seeded ray-cast 2D world with boxes moved between passes)",
    }))


if __name__ == "__main__":
    main()
