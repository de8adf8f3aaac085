#!/usr/bin/env python3
"""bench.py -- ICP edges/sec + ms/GN-iteration on the 5k-node / 20k-edge synthetic graph
(BASELINE.json configs[3]; one GPU runs the whole graph, N GPUs shard its edges).

One step = the hot path over the whole batch, inputs resident in HBM:
  batched ICP of all 20000 edges (+ the covariance block per edge)      [libdpg HIP kernels]
  -> ICP results become BetweenFactor measurements on device
  -> batch Gauss-Newton to convergence (assemble H,b -> [RCCL all-reduce] -> PCG -> retract)
value = ICP edges aligned per second of whole-step wall time (all ranks, max over ranks).

Usage: python bench.py [--gpus N --steps K --warmup W]   (torchrun sets RANK/WORLD_SIZE for N>1)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dpg-slam_amd"))

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
KERNEL_NAME = {"angular": "icp_ang_kernel", "kdtree": "icp_kd_kernel", "grid": "icp_edges_kernel"}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def pmc_traffic(kernel: str):
    """HBM bytes per launch of `kernel` and its SQ-counter fractions from the last committed
    rocprofv3 PMC passes (profiles/pmc_traffic.json, written by tools/pmc_summary.py: (2 x
    FETCH_SIZE + WRITE_SIZE) KiB, the gfx950 correction of MI355X_MICROARCH.md "HBM").  (None, None,
    {}) when no pass covers this kernel."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None, None, {}
    d = json.load(open(path))
    for k, v in d.get("traffic_bytes_per_launch", {}).items():
        if k.split("<")[0] == kernel:
            return float(v), d.get("source"), d.get("sq_fractions", {}).get(k, {})
    return None, None, {}


def kernel_src_sha256() -> str:
    """Content hash of the ICP kernel's sources (the kernel file and the headers it includes): the
    PMC record is stamped with the hash of the sources it profiled (tools/pmc_job.sh), so a stale
    record is visible in the bench line."""
    import hashlib
    h = hashlib.sha256()
    for f in ("dpg_icp_ang.hip", "dpg_icp_tree.h", "dpg_internal.h", "dpg_atan2f.h"):
        h.update(open(os.path.join(ROOT, "dpg-slam_amd", "csrc", f), "rb").read())
    return h.hexdigest()


def pmc_record() -> dict:
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    return json.load(open(path)) if os.path.exists(path) else {}


def host_cpus() -> dict:
    """Core count of this host: the CPUs this process may run on, and lscpu's view of the machine."""
    info = {"affinity": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()}
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in ("CPU(s)", "Model name", "Thread(s) per core"):
                info[k.strip()] = v.strip()
    except Exception:
        pass
    return info


def _median_time(fn, runs: int) -> tuple:
    fn()   # warm-up
    ts = []
    for _ in range(runs):
        t0 = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), out


def cpu_baseline(w, params, sample_edges: int, threads: int = 1, runs: int = 5) -> dict:
    """Oracle (CPU restatement, grid NN) timed on this host, median of `runs` after a warm-up:
    ICP on a bounded random sample of the same workload's edges."""
    from oracle import oracle as O
    rng = np.random.default_rng(0)
    sel = np.sort(rng.choice(w.E, min(sample_edges, w.E), replace=False))
    t, (res, _) = _median_time(lambda: O.icp_batch(w.pts, w.offsets, w.edges[sel], w.est, params, O.NN_GRID, threads),
                               runs)
    return {"icp_edges_per_s": len(sel) / t, "icp_s": t, "n": len(sel), "iters_mean": float(res["iterations"].mean())}


def cpu_gn_baseline(w, icp_results, params, runs: int = 5) -> dict:
    """The oracle's batch Gauss-Newton (block-sparse Cholesky, one thread) on the full graph of the
    same workload from the same initial poses, fed the step's ICP measurements (bit-identical to
    the oracle's own), median of `runs` after a warm-up."""
    from oracle import oracle as O
    F = w.factors_with_icp(icp_results, params)
    X0 = w.est.astype(np.float64)
    t, (_, st) = _median_time(lambda: O.optimize_graph(X0, F), runs)
    return {"ms_per_gn_iter": t * 1e3 / max(1, st.iterations), "gn_iterations": int(st.iterations), "s": t}


def rel_factors(w, V):
    """The graph's factors up to node V with BetweenFactor measurements taken from the estimates
    (est_j in the frame of est_i) -- inputs for TIMING the from-scratch and CPU solves only."""
    from dpgslam import _abi, synth
    E = w.edges[w.edges[:, 1] < V]
    F = np.zeros(V + len(E), _abi.FACTOR_DTYPE)
    F[:V] = w.base_factors[:V]
    F["kind"][V:] = _abi.DPG_FACTOR_BETWEEN
    F["i"][V:], F["j"][V:] = E[:, 0], E[:, 1]
    F["z"][V:] = synth._relative(w.est[E[:, 1]].astype(np.float64), w.est[E[:, 0]].astype(np.float64))
    p = _abi.default_icp_params()
    F["info"][V:] = [1.0 / float(np.float32(p.laser_x_variance)), 1.0 / float(np.float32(p.laser_y_variance)),
                     1.0 / float(np.float32(p.laser_theta_variance))]
    return F


def main_incremental(args):
    """--workload incremental: per-node latency of the incremental path (SURVEY 8f rank 3;
    updatePoseGraphObsConstraints -> optimizeGraph, dpg_slam.cc:255-329) at V = 5000: config 4's
    graph fed node by node.  Node v arrives with its prior/odometry factor, the successive alignment
    (v-1, v) and config 4's loop closures (j, v); each call is ONE dpg_add_node_pairs: the node's
    cloud joins the device scan store, its alignments run as one batched ICP, the factors go into
    the device-resident graph (dpg_inc) and the ISAM2-semantics update runs.  Beside it: round 1's
    per-node cost (dpg_optimize_graph from scratch on the same graph) and the oracle (CPU) per-node
    update on the same call mix at the same size."""
    from dpgslam import _abi, api, synth

    t0 = time.time()
    w = synth.generate(args.config)
    V = min(args.inc_nodes, w.V)
    p = _abi.default_icp_params()
    lc = w.edges[w.n_successive:]
    by_node = [[] for _ in range(V)]
    for k, (j, i) in enumerate(lc):
        if i < V:
            by_node[int(i)].append((int(j), int(i)))
    print(f"generated {args.config} in {time.time() - t0:.1f}s; {sum(len(b) for b in by_node)} loop closures", file=sys.stderr,
          flush=True)

    import ctypes as C
    L = _abi.lib()
    prof, pbuf = [], (C.c_double * 12)()
    lat, icp_ms, sym_ms, num_ms, reord, relin, kept = [], [], [], [], 0, 0, []
    with api.Context(0) as ctx:
        g = api.IncGraph(ctx, mode=args.inc_mode, reorder_every=args.inc_reorder_every,
                         full_refactor=args.inc_full_refactor)
        for v in range(V):
            extra = w.base_factors[v:v + 1]
            ts = time.perf_counter()
            st = g.add_node_pairs(w.cloud(v), w.est[v], np.asarray(by_node[v], np.int32).reshape(-1, 2), extra=extra,
                                  successive=v >= 1, icp_params=p)
            lat.append((time.perf_counter() - ts) * 1e3)
            icp_ms.append(st.ms_icp)
            sym_ms.append(st.update.ms_symbolic)
            num_ms.append(st.update.ms_numeric)
            reord += st.update.reordered
            relin += st.update.relinearized
            kept.append(int(st.update.fronts_kept))
            L.dpg_inc_last_profile(C.c_void_p(g.handle), pbuf, 12)
            prof.append(list(pbuf)[:6] + [pbuf[11]])
            if v % 1000 == 999:
                print(f"node {v + 1}: last latency {lat[-1]:.2f} ms", file=sys.stderr, flush=True)
        X_inc = g.poses()
        nnz = int(st.update.nnz_l)
        n_fac = int(st.update.n_factors)
        # round 1's per-node cost: the whole graph set up and solved from scratch (dpg_optimize_graph)
        ts = time.perf_counter()
        _, gst = ctx.optimize_graph(w.est[:V].astype(np.float64), rel_factors(w, V))
        scratch_ms = (time.perf_counter() - ts) * 1e3
        g.close()

    tail = np.asarray(lat[-500:])
    line = {
        "metric": f"per-node latency of the incremental path at V={V} ({args.config} graph node by node, {args.inc_mode})",
        "unit": "ms/node",
        "p50_ms": float(np.median(tail)), "p90_ms": float(np.percentile(tail, 90)), "mean_ms_all": float(np.mean(lat)),
        "nodes_per_s_tail": float(1e3 / np.mean(tail)),
        "tail_breakdown_ms": {"icp": float(np.mean(icp_ms[-500:])), "symbolic_host": float(np.mean(sym_ms[-500:])),
                              "numeric": float(np.mean(num_ms[-500:])),
                              "symbolic_parts": dict(zip(["incsym", "derive", "lists_upload", "chol_build",
                                                          "chol_host", "chol_upload", "numeric_partial_pick"],
                                                         np.mean(np.asarray(prof[-500:]), 0).round(4).tolist()))},
        "reorders": reord, "relinearized_total": relin, "nnz_L_blocks": nnz, "factors": n_fac,
        # isam_->update's partial re-elimination: updates of the last 500 that kept fronts of the
        # previous factorization, and how many (the others refactored every front: reorders,
        # relinearizations, grown buffers)
        "partial_refactor": {"updates_keeping_fronts_tail": int(np.sum(np.asarray(kept[-500:]) > 0)),
                             "fronts_kept_median_tail": float(np.median(kept[-500:]))},
        "round1_per_node_from_scratch_ms": scratch_ms, "round1_from_scratch_gn_iterations": int(gst.iterations),
    }

    # CPU baseline: the oracle's per-node update at the same size on the same call mix (the graph up to
    # node V - k built in one update, then k single-node updates each with the node's own alignments)
    if args.cpu_nodes > 0:
        from oracle import oracle as O
        k = args.cpu_nodes
        V0 = V - k
        og = O.OracleIncGraph(mode=args.inc_mode)
        og.update(w.est[:V0].astype(np.float64), rel_factors(w, V0))
        cpu = []
        for v in range(V0, V):
            ts = time.perf_counter()
            pf = np.concatenate([og.poses().astype(np.float32), w.est[v:v + 1]])
            pairs = ([(v - 1, v)] if v >= 1 else []) + by_node[v]
            Fv = [w.base_factors[v:v + 1]]
            for q, (a, b) in enumerate(pairs):
                r, _, _ = O.run_icp(w.cloud(b), w.cloud(a), pf[b], pf[a], p, O.NN_GRID)
                if q == 0 or (r.converged and r.status == _abi.DPG_ICP_OK):
                    f = np.zeros(1, _abi.FACTOR_DTYPE)
                    f["kind"], f["i"], f["j"] = _abi.DPG_FACTOR_BETWEEN, a, b
                    f["z"] = np.asarray(r.z, np.float64)
                    f["info"] = [1.0 / float(np.float32(p.laser_x_variance)), 1.0 / float(np.float32(p.laser_y_variance)),
                                 1.0 / float(np.float32(p.laser_theta_variance))]
                    Fv.append(f)
            og.update(w.est[v:v + 1].astype(np.float64), np.concatenate(Fv))
            cpu.append((time.perf_counter() - ts) * 1e3)
        line["cpu_baseline"] = {"value": float(np.median(cpu)), "unit": "ms/node", "cores": 1, "kind": "port",
                                "sample": f"oracle per-node update (ICP grid NN + block-sparse Cholesky, 1 thread) of "
                                          f"nodes {V0}..{V - 1} of the same sequence (graph up to node {V0} built in "
                                          f"one update from estimate-relative measurements), median of {k}"}
    print(json.dumps(line), flush=True)


DPG_BUCKETS = ((0, 1), (1, 10), (10, 50), (50, 1 << 30))


def node_tail(rows):
    """Where the slowest 10 % of the nodes spend their time, against the others: mean wall, node ICP,
    update (symbolic / numeric), executeDPG ms, and the share of updates that reordered, ICP edges
    and submap candidates (per-node rows of the dynamic run)."""
    if not rows:
        return None
    a = np.asarray(rows, np.float64)
    cut = np.percentile(a[:, 0], 90)
    out = {}
    for name, m in (("slowest_10pct", a[:, 0] >= cut), ("others", a[:, 0] < cut)):
        b = a[m]
        out[name] = {"nodes": int(len(b)), "wall_ms": float(b[:, 0].mean()), "icp_ms": float(b[:, 1].mean()),
                     "update_ms": float(b[:, 2].mean()), "symbolic_ms": float(b[:, 3].mean()),
                     "numeric_ms": float(b[:, 4].mean()), "reordered_share": float(b[:, 5].mean()),
                     "icp_edges": float(b[:, 6].mean()), "dpg_ms": float(b[:, 7].mean()),
                     "dpg_candidates": float(b[:, 8].mean())}
    return out


def main_dynamic(args):
    """--workload dynamic: BASELINE config 5 ("10k-node graph with DPG node removal +
    re-linearisation sweep") run through DpgSLAM (dpgslam/slam.py on the GPU backend): 4 passes x
    2500 nodes of a patrol route (synth.make_patrol: 5000-beam 270-degree 30 m scans, noisy
    odometry), ObserveOdometry + ObserveLaser per reading -> per node dpg_add_node (batched ICP of
    the successive + loop-closure alignments, one incremental ISAM2-semantics update) and, from
    pass 1 on, executeDPG (dpg_slam.cc:122-140,865-886); incrementPassNumber -> reoptimize sweep
    at every pass boundary (:25-120), and one more sweep over all 10 000 nodes at the end.
    Reported: nodes/s of the whole run, executeDPG calls/s split by submap-candidate count, the
    sweep times, per-node latency, the map's active-node fraction per pass and the pose error
    against ground truth.  CPU baseline: the oracle replays a fixed sample of the same executeDPG
    calls from the GPU's state before each call (and must reproduce the GPU's counters and state
    exactly), and times the ICP of a sample of the final sweep's edges + the final sweep's solve."""
    import hashlib

    from dpgslam import _abi, api, synth
    from dpgslam.slam import DpgSLAM

    t0 = time.time()
    w = synth.make_patrol(n_passes=args.passes, steps=args.steps_per_pass)
    log(f"generated config5 patrol workload: {w.n_passes} x {w.steps} readings in {time.time() - t0:.1f}s")
    P, N = w.n_passes, w.steps
    sample_k = sorted({0, 1, 2, 3, 50, 500, 1000, 1500, 2000, N - 1} & set(range(N)))
    do_cpu = args.cpu_dpg_calls > 0
    ctx = api.Context(0)
    cp = _abi.default_change_params()
    for kv in args.dpg_param:
        k, v = kv.split("=")
        setattr(cp, k, type(getattr(cp, k))(float(v)) if not isinstance(getattr(cp, k), int) else int(v))
    slam = DpgSLAM(backend="gpu", ctx=ctx, change_params=cp)
    orc, cpu_calls, mismatches = None, [], 0
    if do_cpu:
        from oracle import oracle as O
    node_ms, add_icp_ms, add_upd_ms, dpg, add_split, prof = [], [], [], [], [], []
    node_rows = []   # per node: wall, icp, update, symbolic, numeric, reordered, icp edges, executeDPG ms, candidates
    sweeps, active_end, replay_s, pass_tot = [], [], 0.0, {}
    import ctypes as C
    L, pbuf = _abi.lib(), (C.c_double * 12)()
    amin, amax, rmax = (float(x) for x in w.geom[0])
    t_run = time.perf_counter()
    for p in range(P):
        if p:
            ts = time.perf_counter()
            slam.incrementPassNumber()
            sweeps.append({"before_pass": p, "nodes": len(slam.poses), "factors": int(slam.n_factors),
                           "ms": (time.perf_counter() - ts) * 1e3, "phases_ms": getattr(slam, "last_sweep_ms", None)})
            log(f"pass {p}: sweep over {len(slam.poses)} nodes in {sweeps[-1]['ms']:.0f} ms")
        for k in range(N):
            o = w.odom[p, k]
            rg = w.ranges[p * N + k]
            V0 = len(slam.poses)
            snap = None
            if do_cpu and p >= 1 and k in sample_k and len(cpu_calls) < args.cpu_dpg_calls and slam._store is not None:
                tr = time.perf_counter()
                st_ = slam._dpg_store()
                snap = st_.fetch()
                replay_s += time.perf_counter() - tr
            ts = time.perf_counter()
            slam.ObserveOdometry(o[:2], o[2])
            slam.ObserveLaser(rg, 0.0, rmax, amin, amax)
            dt = (time.perf_counter() - ts) * 1e3
            if len(slam.poses) == V0:
                continue
            node_ms.append(dt)
            la = slam.be.last_add
            add_icp_ms.append(la.ms_icp)
            add_upd_ms.append(la.update.ms_total)
            add_split.append((la.update.ms_symbolic, la.update.ms_numeric))
            dd = slam.last_dpg if p >= 1 else None
            node_rows.append((dt, la.ms_icp, la.update.ms_total, la.update.ms_symbolic, la.update.ms_numeric,
                              int(la.update.reordered), int(la.n_icp_edges), float(dd.ms_total) if dd is not None else 0.0,
                              int(dd.n_candidates) if dd is not None else 0))
            if p == P - 1:   # the last pass: where the symbolic host time goes
                L.dpg_inc_last_profile(C.c_void_p(slam.be.inc.handle), pbuf, 12)
                prof.append(list(pbuf)[:11])
            if p >= 1 and slam.last_dpg is not None:
                d = slam.last_dpg
                dpg.append((int(d.n_candidates), float(d.ms_total), int(d.n_submap_nodes)))
                for key in ("n_removed", "n_added", "n_committed", "n_sectors_deactivated", "n_nodes_deactivated"):
                    pass_tot.setdefault(p, {}).setdefault(key, 0)
                    pass_tot[p][key] += int(getattr(d, key))
            if snap is not None:
                # replay this call on the oracle from the GPU's state before it
                tr = time.perf_counter()
                V1 = len(slam.poses)
                if orc is None:
                    orc = O.OracleDpgStore(np.stack(slam.ranges), np.asarray(slam.geom, np.float32), params=cp)
                elif orc.V < V1:
                    orc.append(np.stack(slam.ranges[orc.V:]), np.asarray(slam.geom[orc.V:], np.float32))
                lab0, sec0, act0 = orc.fetch()   # node V1-1 (the new one) in its initial state
                lab0[:len(snap[0])] = snap[0]
                sec0[:len(snap[1])] = snap[1]
                act0[:len(snap[2])] = snap[2]
                orc.load(lab0, sec0, act0)
                tc = time.perf_counter()
                so = orc.execute_dpg(V1, len(slam.current_pass), slam.poses)
                c_ms = (time.perf_counter() - tc) * 1e3
                go = slam._store.fetch()
                oo = orc.fetch()
                same = so.counters() == slam.last_dpg.counters() and all(
                    hashlib.sha1(a.tobytes()).digest() == hashlib.sha1(b.tobytes()).digest() for a, b in zip(go, oo))
                mismatches += 0 if same else 1
                cpu_calls.append((int(slam.last_dpg.n_candidates), c_ms, same))
                replay_s += time.perf_counter() - tr
            if len(node_ms) % 500 == 0:
                log(f"pass {p} node {len(slam.poses)}: node {node_ms[-1]:.1f} ms, dpg {dpg[-1][1] if dpg else 0:.2f} ms "
                    f"({dpg[-1][0] if dpg else 0} candidates)")
        if p >= 1:
            _, _, act = slam._store.fetch()
            active_end.append({"pass": p, "active_fraction": float(act.mean()),
                               "past_active_fraction": float(act[:int(np.sum(slam.node_pass < p))].mean()),
                               **pass_tot.get(p, {})})
    if args.dump_pairs:   # the graph's node pairs in arrival order, for offline ordering studies
        L.dpg_inc_pairs.restype = C.c_int64
        hdl = C.c_void_p(slam.be.inc.handle)
        npairs = L.dpg_inc_pairs(hdl, None, None, C.c_int64(0))
        lo, hi = np.zeros(npairs, np.int32), np.zeros(npairs, np.int32)
        L.dpg_inc_pairs(hdl, lo.ctypes.data_as(C.c_void_p), hi.ctypes.data_as(C.c_void_p), C.c_int64(npairs))
        np.savez_compressed(args.dump_pairs, lo=lo, hi=hi)
    # the sweep at 10k nodes (incrementPassNumber after the last pass)
    est_final = slam.poses.copy()
    ts = time.perf_counter()
    slam.reoptimize()
    sweeps.append({"before_pass": P, "nodes": len(slam.poses), "factors": int(slam.n_factors),
                   "ms": (time.perf_counter() - ts) * 1e3, "phases_ms": getattr(slam, "last_sweep_ms", None)})
    wall = time.perf_counter() - t_run - replay_s
    V = len(slam.poses)
    # pose error against ground truth (map frame = pass 0's start)
    gtm = w.gt_map().reshape(-1, 3)
    created = np.asarray(slam.node_pass)
    err = None
    if V == P * N:
        e = slam.poses[:, :2].astype(np.float64) - gtm[:, :2]
        err = {"rms_m": float(np.sqrt((e ** 2).sum(1).mean())), "max_m": float(np.sqrt((e ** 2).sum(1)).max())}
        # what the change detection sees: each later-pass node against the nearest pass-0 node (by
        # ground truth), relative pose estimated vs true
        from scipy.spatial import cKDTree
        n0 = int(np.sum(created == 0))
        _, jn = cKDTree(gtm[:n0, :2]).query(gtm[n0:, :2])
        rel_e = synth._relative(slam.poses[n0:].astype(np.float64), slam.poses[jn].astype(np.float64))
        rel_t = synth._relative(gtm[n0:], gtm[jn])
        dd = rel_e - rel_t
        err["cross_pass_rel_rms_m"] = float(np.sqrt((dd[:, :2] ** 2).sum(1).mean()))
        err["cross_pass_rel_rms_rad"] = float(np.sqrt((np.arctan2(np.sin(dd[:, 2]), np.cos(dd[:, 2])) ** 2).mean()))
    dpg_a = np.asarray(dpg, np.float64).reshape(-1, 3)
    buckets = []
    for lo, hi in DPG_BUCKETS:
        m = (dpg_a[:, 0] >= lo) & (dpg_a[:, 0] < hi)
        if m.any():
            ms = float(dpg_a[m, 1].mean())
            bk = {"candidates": f"[{lo},{hi if hi < 1 << 30 else 'inf'})", "calls": int(m.sum()), "ms_per_call": ms,
                  "calls_per_s": 1e3 / ms}
            cm = [c for c in cpu_calls if lo <= c[0] < hi]
            if cm:
                bk["cpu_ms_per_call"] = float(np.mean([c[1] for c in cm]))
                bk["cpu_calls"] = len(cm)
            buckets.append(bk)
    line = {
        "metric": "config5 DpgSLAM run: nodes/s (per-node ICP + incremental solve + executeDPG, sweeps at pass "
                  "boundaries); executeDPG calls/s by candidate count; sweep ms",
        "value": V / wall, "unit": "nodes/s", "higher_is_better": True, "n_gpus": 1,
        "config": {"workload": f"config5: {P} passes x {N} readings of a serpentine patrol route through a "
                               f"16x16-room building (5000-beam 270-degree 30 m scans, 2 mm range noise, 64 movable "
                               f"boxes), DpgSLAM defaults", "nodes": V},
        "data": "synthetic (seeded ray-cast building, boxes added/removed between passes, noisy odometry)",
        "wall_s": wall, "nodes_per_pass": [int(np.sum(created == q)) for q in range(P)],
        "node_tail": node_tail(node_rows),
        "node_ms": {"p50": float(np.median(node_ms)), "p90": float(np.percentile(node_ms, 90)),
                    "mean": float(np.mean(node_ms)), "icp_mean": float(np.mean(add_icp_ms)),
                    "update_mean": float(np.mean(add_upd_ms)),
                    "update_symbolic_mean": float(np.mean([a for a, _ in add_split])),
                    "update_numeric_mean": float(np.mean([b for _, b in add_split])),
                    "last_pass_symbolic_parts": dict(zip(("incsym", "derive", "lists_upload", "chol_build", "chol_host",
                                                          "chol_upload", "factor_mflop", "max_front_blocks",
                                                          "fused_fraction", "supernodes", "levels"),
                                                         np.round(np.mean(prof, 0), 4).tolist()))
                    if prof else None,
                    "end_factor": dict(zip(("mflop", "max_front_blocks", "fused", "supernodes", "levels"), prof[-1][6:11]))
                    if prof else None},
        "dpg": {"calls": len(dpg_a), "ms_per_call": float(dpg_a[:, 1].mean()) if len(dpg_a) else None,
                "calls_per_s": float(1e3 / dpg_a[:, 1].mean()) if len(dpg_a) else None,
                # the reference's sector rule collapses the past map on this route: most calls
                # see an empty submap, so the rate over the calls with >= 1 candidate stands beside it
                "calls_ge1_candidate": int((dpg_a[:, 0] >= 1).sum()) if len(dpg_a) else 0,
                "calls_per_s_ge1_candidate": float(1e3 / dpg_a[dpg_a[:, 0] >= 1, 1].mean())
                if len(dpg_a) and (dpg_a[:, 0] >= 1).any() else None,
                "candidates_mean": float(dpg_a[:, 0].mean()) if len(dpg_a) else None,
                "submap_nodes_mean": float(dpg_a[:, 2].mean()) if len(dpg_a) else None, "by_candidates": buckets},
        "sweeps": sweeps, "active": active_end, "pose_error_vs_gt": err,
    }
    if do_cpu:
        sp = api.Context  # noqa: F841 (keeps the import order explicit)
        cb = {"value": float(1e3 / np.mean([c[1] for c in cpu_calls])) if cpu_calls else None,
              "unit": "executeDPG calls/s", "cores": 1, "kind": "port",
              "sample": f"oracle (C++ restatement, 1 thread) replaying {len(cpu_calls)} of the run's executeDPG calls "
                        f"(readings {sample_k} of passes 1..{P - 1}) from the GPU's state before each call; "
                        f"{len(cpu_calls) - mismatches} of {len(cpu_calls)} reproduce the GPU's counters and state "
                        f"bit for bit",
              "replay_bit_exact": mismatches == 0}
        # the final sweep's ICP (a sample of its edges) and its solve on the oracle
        lc = ctx.loop_closure_candidates(est_final, slam.node_pass, 5.0, 2.0)
        rng = np.random.default_rng(0)
        sel = lc[np.sort(rng.choice(len(lc), min(args.cpu_sample, len(lc)), replace=False))] if len(lc) else lc
        pts, offs = slam._clouds()
        p_icp = _abi.default_icp_params()
        t, _ = _median_time(lambda: O.icp_batch(pts, offs, sel, est_final, p_icp, O.NN_GRID, 1), 3)
        og = O.OracleIncGraph()
        tg = time.perf_counter()
        og.update(est_final.astype(np.float64), slam.factors)
        cb["sweep_icp_edges_per_s"] = len(sel) / t
        cb["sweep_solve_ms"] = (time.perf_counter() - tg) * 1e3
        cb["sweep_sample"] = (f"oracle ICP (grid NN, 1 thread) on {len(sel)} random loop-closure edges of the final "
                              f"sweep, median of 3; oracle solve of the final sweep's graph ({len(slam.factors)} factors)")
        line["cpu_baseline"] = cb
    print(json.dumps(line), flush=True)
    ctx.close()


def main_dpg(args):
    """--workload dpg: executeDPG (dpg_slam.cc:865-886) at config-5 scale on a map that does not
    collapse: 4 passes x 2500 nodes of a 64 m building (make_dynamic: 5000-beam 270-degree 30 m
    noise-free scans, 48 movable boxes flipping between passes), every pass starting at the same
    pose, node poses = ground truth, executeDPG after every node of passes 1..3 in order.  (With
    estimated poses or range noise the reference's rules deactivate nearly every past node within
    a pass -- see the dynamic workload and DESIGN.md; here 40-90 % stay active.)  Reported: calls/s
    overall and split by submap-candidate count, per pass.  CPU baseline: after the timed run the
    sequence is replayed on the GPU and, before a stratified sample of calls (spread over the
    candidate buckets), the oracle takes over from the GPU's state, times the call and must
    reproduce the GPU's counters and state bit for bit."""
    import hashlib

    from dpgslam import api, synth

    t0 = time.time()
    w = synth.make_dynamic(n_passes=args.passes, nodes_per_pass=args.steps_per_pass, world_size=64.0, fov_deg=270.0,
                           n_boxes=48, range_noise=0.0)
    log(f"generated the DPG workload: {w.V} nodes in {time.time() - t0:.1f}s")
    ctx = api.Context(0)
    calls = list(range(int(w.pass_start[1]), w.V))

    def run(g, on_call=None):
        out = []
        for q, v in enumerate(calls):
            p = int(w.pass_of[v])
            if on_call is not None:
                on_call(q, v, g)
            st = g.execute_dpg(v + 1, int(v - w.pass_start[p] + 1), w.est[:v + 1])
            out.append((int(st.n_candidates), float(st.ms_total), int(st.n_submap_nodes), p, st.counters()))
            if q % 1000 == 999:
                log(f"call {q + 1}/{len(calls)}: {st.ms_total:.2f} ms, {st.n_candidates} candidates")
        return out

    g = api.DpgStore(ctx, w.ranges, w.geom)
    run(g)                       # warm-up pass over the whole sequence on a throw-away store
    g.close()
    g = api.DpgStore(ctx, w.ranges, w.geom)
    ctx.synchronize()
    t1 = time.perf_counter()
    rec = run(g)
    wall = time.perf_counter() - t1
    _, _, act = g.fetch()
    g.close()
    cand = np.asarray([r[0] for r in rec])
    ms = np.asarray([r[1] for r in rec])
    passes = np.asarray([r[3] for r in rec])
    buckets = []
    for lo, hi in DPG_BUCKETS:
        m = (cand >= lo) & (cand < hi)
        if m.any():
            buckets.append({"candidates": f"[{lo},{hi if hi < 1 << 30 else 'inf'})", "calls": int(m.sum()),
                            "ms_per_call": float(ms[m].mean()), "calls_per_s": float(1e3 / ms[m].mean())})
    per_pass = []
    for p in range(1, args.passes):
        m = passes == p
        last = int(w.pass_start[p + 1]) if p + 1 < len(w.pass_start) else w.V
        per_pass.append({"pass": p, "calls": int(m.sum()), "calls_per_s": float(1e3 / ms[m].mean()),
                         "candidates_mean": float(cand[m].mean()), "calls_ge50": float((cand[m] >= 50).mean())})
    line = {
        "metric": "executeDPG calls/s at config-5 scale (10k-node 4-pass dynamic map), split by submap-candidate count",
        "value": len(calls) / wall, "unit": "calls/s", "higher_is_better": True, "n_gpus": 1,
        "ms_per_call": 1e3 * wall / len(calls), "calls": len(calls),
        "config": {"workload": f"config5 DPG: {args.passes} passes x {args.steps_per_pass} nodes, 64 m building, "
                               f"5000-beam 270-degree 30 m noise-free scans, 48 movable boxes, ground-truth poses, "
                               f"executeDPG after every node of passes 1..{args.passes - 1}", "nodes": int(w.V)},
        "data": "synthetic (seeded ray-cast building, boxes added/removed between passes)",
        "by_candidates": buckets, "per_pass": per_pass,
        "past_active_fraction_end": float(act[:int(w.pass_start[args.passes - 1])].mean()),
    }
    if args.cpu_dpg_calls > 0:
        from oracle import oracle as O
        rng = np.random.default_rng(1)
        pick = set()
        per_b = max(1, args.cpu_dpg_calls // len(DPG_BUCKETS))
        for lo, hi in DPG_BUCKETS:
            idx = np.nonzero((cand >= lo) & (cand < hi))[0]
            if len(idx):
                pick.update(int(i) for i in rng.choice(idx, min(per_b, len(idx)), replace=False))
        orc = O.OracleDpgStore(w.ranges, w.geom)
        res = []

        def replay(q, v, gs):
            if q not in pick:
                return
            snap = gs.fetch()
            orc.load(*snap)
            p = int(w.pass_of[v])
            tc = time.perf_counter()
            so = orc.execute_dpg(v + 1, int(v - w.pass_start[p] + 1), w.est[:v + 1])
            c_ms = (time.perf_counter() - tc) * 1e3
            res.append((q, int(so.n_candidates), c_ms, so.counters(), orc.fetch()))

        g = api.DpgStore(ctx, w.ranges, w.geom)
        posts = {}

        def hook(q, v, gs):
            if q - 1 in pick:   # the GPU's state after the picked call
                posts[q - 1] = [hashlib.sha1(a.tobytes()).digest() for a in gs.fetch()]
            replay(q, v, gs)

        rec2 = run(g, hook)
        last = len(calls) - 1
        if last in pick:
            posts[last] = [hashlib.sha1(a.tobytes()).digest() for a in g.fetch()]
        g.close()
        ok = 0
        for q, nc, c_ms, cnt, st in res:
            same = cnt == rec2[q][4] and [hashlib.sha1(a.tobytes()).digest() for a in st] == posts.get(q)
            ok += int(same)
        cb_b = []
        for lo, hi in DPG_BUCKETS:
            sel = [r for r in res if lo <= r[1] < hi]
            if sel:
                cb_b.append({"candidates": f"[{lo},{hi if hi < 1 << 30 else 'inf'})", "calls": len(sel),
                             "cpu_ms_per_call": float(np.mean([r[2] for r in sel]))})
        # the CPU rate of the whole sequence, weighting each bucket's mean by its share of the calls
        tot = sum(b["calls"] for b in buckets)
        cpu_ms = sum(b["calls"] / tot * next(c["cpu_ms_per_call"] for c in cb_b if c["candidates"] == b["candidates"])
                     for b in buckets if any(c["candidates"] == b["candidates"] for c in cb_b))
        line["cpu_baseline"] = {"value": 1e3 / cpu_ms if cpu_ms else None, "unit": "calls/s", "cores": 1, "kind": "port",
                                "sample": f"oracle (C++ restatement, 1 thread) taking over from the GPU's state before "
                                          f"{len(res)} calls stratified over the candidate buckets; bucket means "
                                          f"weighted by the run's call mix; {ok} of {len(res)} reproduce the GPU's "
                                          f"counters and state bit for bit",
                                "by_candidates": cb_b, "replay_bit_exact": ok == len(res)}
    print(json.dumps(line), flush=True)
    ctx.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="config4")
    ap.add_argument("--cpu-sample", type=int, default=500, help="edges in the CPU-baseline ICP sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI; gloo only to rehearse "
                         "the multi-rank path on fewer GPUs than ranks)")
    ap.add_argument("--icp-variant", default="angular", choices=["angular", "kdtree", "grid"],
                    help="nearest-neighbour machinery of the ICP kernel (results are identical)")
    ap.add_argument("--shard", default="interleave", choices=["interleave", "contiguous"],
                    help="N > 1: ICP edge shares (dpgslam.dist.plan)")
    ap.add_argument("--dump-pairs", default=None, help="dynamic: save the graph's node pairs (npz) after the run")
    ap.add_argument("--refactor-delta", type=float, default=None,
                    help="dpg_gn_params.refactor_delta: chord steps (reuse the Cholesky factor) once max|delta| is below it")
    ap.add_argument("--workload", default="batch", choices=["batch", "incremental", "dynamic", "dpg"],
                    help="batch: the headline step (all edges + GN); incremental: per-node latency of "
                         "dpg_add_node_pairs at V = 5000 (1 GPU); dynamic: config 5 through DpgSLAM (1 GPU); dpg: executeDPG at config-5 "
                         "scale on a map that does not collapse (1 GPU)")
    ap.add_argument("--passes", type=int, default=4)
    ap.add_argument("--steps-per-pass", type=int, default=2500)
    ap.add_argument("--cpu-dpg-calls", type=int, default=30, help="executeDPG calls replayed on the oracle")
    ap.add_argument("--dpg-param", action="append", default=[],
                    help="DpgParameters override, e.g. occ_grid_resolution=0.1 or num_sectors=8 (repeatable)")
    ap.add_argument("--dist", default="native", choices=["native", "torch"],
                    help="under torchrun: native = libdpg's rank form (its own RCCL communicator, the "
                         "pipelined GN); torch = the per-rank step API + Python GN loop over torch.distributed")
    ap.add_argument("--virtual", type=int, default=0,
                    help="K > 0: K virtual devices on one card (dpg_ctx_create_virtual) -- a rehearsal of "
                         "the sharded paths, not a scaling number")
    ap.add_argument("--kernel-variant", type=int, default=0,
                    help="diagnostic A/B: the angular ICP kernel's form (dpg_ctx_set_icp_kernel_variant; 0 = default)")
    ap.add_argument("--schedule", default="measured", choices=["measured", "caller"],
                    help="batched ICP dispatch (dpg_ctx_set_icp_schedule); results are identical")
    ap.add_argument("--inc-mode", default="isam2", choices=["isam2", "batch"])
    ap.add_argument("--inc-nodes", type=int, default=5000)
    ap.add_argument("--inc-reorder-every", type=int, default=32, help="incremental: a fresh order every this many nodes")
    ap.add_argument("--inc-full-refactor", action="store_true", help="incremental: refactor every front every update")
    ap.add_argument("--cpu-nodes", type=int, default=8, help="nodes in the incremental CPU-baseline sample")
    args = ap.parse_args()
    if args.workload == "incremental":
        return main_incremental(args)
    if args.workload == "dynamic":
        return main_dynamic(args)
    if args.workload == "dpg":
        return main_dpg(args)

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist
    from dpgslam import _abi, api, synth
    from dpgslam import dist as D

    # The forms of one job:
    #   single  -- N = 1: one device context;
    #   multi   -- N > 1 without a launcher: ONE process over N devices (dpg_ctx_create_multi: sharded
    #              ICP, the pipelined GN with an in-stream ncclAllReduce per iteration);
    #   rank    -- under torchrun (WORLD_SIZE = N): one process per GPU, each a rank of one RCCL
    #              communicator made inside libdpg (dpg_ctx_create_rank), the same native paths;
    #   virtual -- --virtual K: K virtual devices on one card (rehearsal of the sharded paths);
    #   torch   -- --dist torch under torchrun: round 2's Python GN loop over torch.distributed.
    n_vis = torch.cuda.device_count()
    if world > 1:
        mode = "torch" if args.dist == "torch" else "rank"
        if world != args.gpus:
            log(f"warning: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE")
    elif args.virtual:
        mode = "virtual"
    elif args.gpus > 1:
        mode = "multi"
        if n_vis < args.gpus:
            log(f"error: --gpus {args.gpus} asked, {n_vis} GPU(s) visible")
            sys.exit(2)
    else:
        mode = "single"
    if mode == "torch":
        return main_torch_dist(args, rank, world, local_rank)

    gpu = local_rank % max(1, n_vis)   # == local_rank on a full node
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        dist.init_process_group("gloo")   # host-side barrier / id hand-off; the data path is libdpg's RCCL
    t0 = time.time()
    w = synth.generate(args.config)
    log(f"[rank {rank}] generated {args.config}: V={w.V} E={w.E} points={len(w.pts)} in {time.time() - t0:.1f}s")
    params = _abi.default_icp_params()
    gp = _abi.default_gn_params()
    if args.refactor_delta is not None:
        gp.refactor_delta = args.refactor_delta

    if mode == "rank":
        obj = [api.nccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        ctx = api.Context(gpu, rank=(obj[0], rank, world))
    elif mode == "multi":
        ctx = api.Context(0, n_gpus=args.gpus)
    elif mode == "virtual":
        ctx = api.Context(gpu, virtual=args.virtual)
    else:
        ctx = api.Context(gpu)
        ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    n_gpus = {"single": 1, "multi": args.gpus, "rank": world, "virtual": 1}[mode]
    ctx.set_icp_variant(args.icp_variant)
    ctx.set_icp_schedule(args.schedule)
    if args.kernel_variant:
        ctx.set_icp_kernel_variant(args.kernel_variant)
    # one-off cost of a solve: the host->device upload of the clouds, the edge staging
    # (icp_prepare: guesses + edge records) and the GN setup (ordering, symbolic analysis, Cholesky
    # plan) are outside the repeated step; each is timed here to its end on the device
    t0 = time.perf_counter()
    ctx.upload_scans(w.pts, w.offsets, params.downsample_icp_points_ratio)
    ctx.synchronize()
    t1 = time.perf_counter()
    ctx.icp_prepare(w.edges, w.est, params)   # ALL edges: a multi-device context shards them itself
    ctx.synchronize()
    t2 = time.perf_counter()
    F = w.factors_placeholder()
    ctx.gn_setup(w.V, F, params=gp)
    ctx.synchronize()
    t3 = time.perf_counter()
    setup = {"upload_ms": (t1 - t0) * 1e3, "icp_prepare_ms": (t2 - t1) * 1e3, "gn_setup_ms": (t3 - t2) * 1e3,
             "gn_setup_parts_ms": ctx.gn_setup_profile()}
    X0 = w.est.astype(np.float64)

    def step():
        ctx.icp_run(compute_cov=True)
        ctx.gn_take_icp(w.icp_factor_first, w.E, w.n_successive, params)   # on the device(s) that aligned them
        ctx.gn_set_poses(X0)
        return ctx.gn_run()[0]

    def barrier():
        ctx.synchronize()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    # cold: the first run knows no alignment costs, so it dispatches in the caller's order -- what a
    # one-off batch gets; the headline's measured schedule (LPT + longest first) is learnt from it
    cold = {}
    for k in range(args.warmup):
        st = step()
        if k == 0:
            ctx.synchronize()
            cold["icp_kernel_ms_first_run"] = ctx.icp_kernel_ms()
    if args.schedule == "measured" and args.warmup > 0:
        # the caller's order again, warm, beside the measured one (same results; untimed)
        ctx.set_icp_schedule("caller")
        ctx.icp_prepare(w.edges, w.est, params)
        cms = []
        for _ in range(3):
            step()
            ctx.synchronize()
            cms.append(ctx.icp_kernel_ms())
        cold["icp_kernel_ms_caller_order"] = float(np.median(cms))
        ctx.set_icp_schedule("measured")
        ctx.icp_prepare(w.edges, w.est, params)   # every cost known: planned at once
        step()
    barrier()
    icp_ms, cov_ms, idx_ms, gn_iters, gn_ms, n_fact = [], [], [], [], [], []
    t_start = time.perf_counter()
    for _ in range(args.steps):
        ts = time.perf_counter()
        st = step()
        ctx.synchronize()
        icp_ms.append(ctx.icp_kernel_ms())
        cov_ms.append(ctx.cov_kernel_ms())
        idx_ms.append(ctx.kdtree_build_ms())
        gn_iters.append(st["iterations"])
        n_fact.append(ctx.gn_factorizations())
        # the covariance runs beside the GN on its own stream (dpg_cov_batch_overlapped): then it is
        # not part of the step's serial time and is not taken off the GN's share
        cov_serial = 0.0 if ctx.cov_overlapped() else cov_ms[-1]
        gn_ms.append((time.perf_counter() - ts) * 1e3 - icp_ms[-1] - cov_serial - idx_ms[-1])
    barrier()
    elapsed = time.perf_counter() - t_start

    def reduce(vals, op):
        if world == 1:
            return vals
        t = torch.tensor(vals, dtype=torch.float64)
        dist.all_reduce(t, op=op)
        return t.tolist()

    elapsed = reduce([elapsed], dist.ReduceOp.MAX if world > 1 else None)[0]
    ms_step = elapsed * 1e3 / args.steps
    algo_bytes = reduce([ctx.icp_algorithmic_bytes()], dist.ReduceOp.SUM if world > 1 else None)[0]
    k_ms, gn_it_ms = reduce([float(np.mean(icp_ms)), float(np.mean(gn_ms) / max(1.0, np.mean(gn_iters)))],
                            dist.ReduceOp.MAX if world > 1 else None)
    # one launch per device: the aggregate algorithmic rate against the devices' aggregate peak
    achieved = algo_bytes / (k_ms * 1e-3) / 1e9
    ck = sorted(cold)
    cold_red = dict(zip(ck, reduce([cold[k] for k in ck], dist.ReduceOp.MAX if world > 1 else None))) if ck else {}
    res, _ = ctx.icp_fetch(with_hessian=False)   # a collective on the rank form
    cold_solve = None
    if mode == "single":
        cold_solve = cold_single_solve(api, w, params, gp, gpu)
    stats = {"icp_kernel_ms": k_ms, "cov_kernel_ms": float(np.mean(cov_ms)), "index_build_ms": float(np.mean(idx_ms)),
             "gn_iterations": float(np.mean(gn_iters)), "gn_factorizations": float(np.mean(n_fact)),
             "ms_per_gn_iter": gn_it_ms,
             "icp_iters_mean": float(res["iterations"].mean()), "icp_iters_max": int(res["iterations"].max()),
             "final_error": st["final_error"], "pcg_iterations": st["pcg_iterations"], "gn_loop": "native"}
    cpu = None
    if rank == 0 and mode == "single" and not args.no_cpu_baseline:
        cores = host_cpus()
        cb = cpu_baseline(w, params, args.cpu_sample, threads=1)
        gnb = cpu_gn_baseline(w, res, params)
        cpu = {"value": cb["icp_edges_per_s"], "unit": "edges/s", "cores": 1, "kind": "port",
               "sample": f"oracle (C restatement, grid NN, 1 thread) ICP on {cb['n']} random edges of "
                         f"{args.config}: median of 5 runs after a warm-up ({cb['icp_s']:.2f} s per run, mean "
                         f"{cb['iters_mean']:.1f} ICP iterations)",
               "gn_ms_per_iter": gnb["ms_per_gn_iter"],
               "gn_sample": f"oracle batch GN (block-sparse Cholesky, 1 thread) on the full {args.config} graph, "
                            f"{gnb['gn_iterations']} iterations, median of 5 runs ({gnb['s']:.2f} s per solve)",
               "host": cores}
        # the same ICP sample over edges with OpenMP on the lease's CPU share: the GPU
        # box exposes every host CPU in the affinity mask (256) but one GPU's lease is 16 of them
        # (OMP_NUM_THREADS=16 there; the pool's rules cap worker pools at the share)
        share = int(os.environ.get("OMP_NUM_THREADS") or 0) or 16
        nt = max(1, min(share, cores.get("affinity") or 1))
        if nt > 1:
            cm = cpu_baseline(w, params, args.cpu_sample, threads=nt)
            cpu["multithread"] = {"value": cm["icp_edges_per_s"], "unit": "edges/s", "cores": nt,
                                  "share_rule": f"the GPU lease's CPU share: {nt} threads (OMP_NUM_THREADS on the "
                                                f"box) of the {cores.get('affinity')} CPUs in the affinity mask",
                                  "sample": f"same sample, OpenMP over edges, median of 5 runs ({cm['icp_s']:.2f} s per run)"}

    traffic, traffic_src, sq = pmc_traffic(KERNEL_NAME[args.icp_variant])
    if mode != "single":   # the PMC pass measured the whole 1-GPU launch; a device's launch holds only its shard
        traffic, traffic_src, sq = None, None, {}
    # the PMC record's provenance, and the kernel against the limiters the counters name: VALU issue
    # (wave64 VALU = 2 cycles on a SIMD-32, 1024 SIMDs at 2.4 GHz) and the LDS array (one access
    # cycle per CU per clock, SQ_LDS_IDX_ACTIVE), per launch from the PMC record over this run's
    # kernel time
    rec = pmc_record()
    src_now = kernel_src_sha256()
    pmc_meta = {"record": traffic_src, "src_sha256": rec.get("src_sha256"), "git_sha": rec.get("git_sha"),
                "matches_running_kernel": rec.get("src_sha256") == src_now}
    counts = next((v for k, v in rec.get("counts", {}).items() if k.split("<")[0] == KERNEL_NAME[args.icp_variant]), {})
    limiters = []
    if counts and mode == "single":
        t = k_ms * 1e-3
        if counts.get("SQ_INSTS_VALU"):
            a = counts["SQ_INSTS_VALU"] / t
            limiters.append({"bound": "valu_issue", "achieved": a, "peak": 1024 * 2.4e9 / 2, "unit": "wave-instr/s",
                             "frac": a / (1024 * 2.4e9 / 2)})
        if counts.get("SQ_LDS_IDX_ACTIVE"):
            a = counts["SQ_LDS_IDX_ACTIVE"] / t
            limiters.append({"bound": "lds_array", "achieved": a, "peak": 256 * 2.4e9, "unit": "LDS cycles/s",
                             "frac": a / (256 * 2.4e9),
                             "bank_conflict_cycles_per_lds_instr": counts.get("SQ_LDS_BANK_CONFLICT", 0.0) /
                             max(1.0, counts.get("SQ_INSTS_LDS", 0.0))})
    if rank == 0:
        line = {
            "metric": "ICP edges/sec + ms/GN-iter on 5k-node/20k-edge synthetic graph, 1->8 GPU",
            "value": w.E * args.steps / elapsed,
            "unit": "edges/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "fp32 (ICP) + fp64 (GN)",
            "data": "synthetic (seeded ray-cast 2D world, 5000-beam scans -> ~1000-pt clouds)",
            "config": {"workload": f"{args.config}: {w.V} nodes / {w.E} ICP edges / {len(F)} factors, "
                                   f"~{int(np.mean(np.diff(w.offsets)) / 5)}-pt downsampled scans",
                       "nodes": w.V, "icp_edges": w.E, "factors": len(F),
                       "parallelism": f"edge-sharded dp{ctx.n_ranks}" + ("" if mode == "single" else f" ({mode} form)")},
            "form": mode, "ranks": ctx.n_ranks, "icp_schedule": args.schedule,
            "ms_per_gn_iter": stats["ms_per_gn_iter"],
            "gn_iterations": stats["gn_iterations"],
            "gn_factorizations": stats["gn_factorizations"],
            "gn_loop": stats["gn_loop"],
            "final_error": stats["final_error"],
            "icp_kernel_ms": stats["icp_kernel_ms"],
            **{k: v for k, v in cold_red.items()},
            "setup_ms": setup["upload_ms"] + setup["icp_prepare_ms"] + setup["gn_setup_ms"], "setup": setup,
            **({"cold_single_solve_ms": cold_solve["total_ms"], "cold_single_solve": cold_solve} if cold_solve else {}),
            "cold_note": "icp_kernel_ms_first_run: the first warm-up step (no learnt costs: the caller's order, "
                         "the first launch after the upload); icp_kernel_ms_caller_order: the caller's order "
                         "again after the warm-up (median of 3, untimed); icp_kernel_ms: the timed steps on the "
                         "measured schedule (LPT + longest first from the warm-up's iteration counts)",
            "cov_kernel_ms": stats["cov_kernel_ms"],
            "cov_beside_gn": ctx.cov_overlapped(),
            "index_build_ms": stats["index_build_ms"],
            "icp_variant": args.icp_variant,
            "icp_edges_per_s_kernel": w.E / (stats["icp_kernel_ms"] * 1e-3),
            "icp_iters_mean": stats["icp_iters_mean"],
            "icp_iters_max": stats["icp_iters_max"],
            "gn_note": "ms_per_gn_iter averages plain GN steps and chord steps that reuse the last Cholesky "
                       "factor (gn_factorizations of gn_iterations refactor; DESIGN.md section 3)",
            # roofline of the dominant kernel against HBM (SURVEY 8d's algorithmic bytes); the counters
            # say what actually limits it: "limiter" + the SQ fractions of the last committed PMC pass
            "roofline": {"bound": "hbm", "achieved": achieved if mode != "virtual" else None,
                         "peak": HBM_PEAK_GBS * n_gpus, "unit": "GB/s",
                         "frac": achieved / (HBM_PEAK_GBS * n_gpus) if mode != "virtual" else None,
                         **({"note": "virtual form: the K shares time-share ONE card and each share's events "
                                     "bracket only its own kernel, so no per-launch time bounds the union; "
                                     "no fraction is reported"} if mode == "virtual" else {}),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": KERNEL_NAME[args.icp_variant] + " (correspondence search + fit, fused)",
                         "bytes_per_launch": algo_bytes,
                         "limiter": "VALU issue + LDS latency with per-iteration workgroup barriers, not HBM: "
                                    "the clouds stay in LDS for all iterations (traffic << algorithmic bytes)",
                         **({"sq": sq} if sq else {}), "pmc": pmc_meta, "kernel_src_sha256": src_now},
            "roofline_limiters": limiters,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    ctx.close()


def cold_single_solve(api, w, params, gp, gpu):
    """A one-off batched solve on a FRESH context, timed end to end on the host clock: the clouds'
    upload, icp_prepare, the first ICP run (caller's order, the angle index built), the GN setup,
    the ICP factors taken on the device, and the GN to convergence (dpg_slam.cc:35-120: every
    reoptimize builds its graph afresh).  The repeated step of the headline excludes all but the
    last three; this is what a single solve costs."""
    X0 = w.est.astype(np.float64)
    ph = {}
    tc = time.perf_counter()
    with api.Context(gpu) as c:
        c.synchronize()
        t0 = time.perf_counter()
        c.upload_scans(w.pts, w.offsets, params.downsample_icp_points_ratio)
        c.icp_prepare(w.edges, w.est, params)
        c.synchronize()
        t1 = time.perf_counter()
        c.icp_run(compute_cov=True)
        ta = time.perf_counter()
        F = w.factors_placeholder()
        c.gn_setup(w.V, F, params=gp)   # host work while the GPU aligns
        tb = time.perf_counter()
        c.synchronize()
        t2 = time.perf_counter()
        c.gn_take_icp(w.icp_factor_first, w.E, w.n_successive, params)
        c.gn_set_poses(X0)
        st = c.gn_run()[0]
        c.synchronize()
        t3 = time.perf_counter()
        ph = {"total_ms": (t3 - t0) * 1e3, "ctx_create_ms": (t0 - tc) * 1e3, "upload_prepare_ms": (t1 - t0) * 1e3,
              "icp_and_gn_setup_ms": (t2 - t1) * 1e3, "gn_ms": (t3 - t2) * 1e3,
              "icp_run_call_ms": (ta - t1) * 1e3, "gn_setup_call_ms": (tb - ta) * 1e3, "wait_ms": (t2 - tb) * 1e3,
              "icp_kernel_ms": c.icp_kernel_ms(), "index_build_ms": c.kdtree_build_ms(),
              "gn_iterations": st["iterations"], "final_error": st["final_error"],
              "note": "fresh context: upload + prepare -> ICP (caller's order, index built) with the GN "
                      "setup on the host meanwhile -> GN to convergence; host clock to the device's end "
                      "(ctx_create_ms: the context's creation before it, its streams included)"}
    return ph


def main_torch_dist(args, rank, world, local_rank):
    """--dist torch under torchrun: one process per GPU, the per-rank step API of libdpg and the
    Python GN loop (dpgslam.dist.gn_loop) with torch.distributed's all-reduce (RCCL) of the packed
    system per iteration -- round 2's form, kept as the alternative to the native rank form."""
    import torch
    import torch.distributed as dist
    from dpgslam import _abi, api, synth
    from dpgslam import dist as D

    gpu = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if args.backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)   # RCCL over xGMI
    else:
        dist.init_process_group("gloo")
    w = synth.generate(args.config)
    params = _abi.default_icp_params()
    gp = _abi.default_gn_params()
    if args.refactor_delta is not None:
        gp.refactor_delta = args.refactor_delta
    ctx = api.Context(gpu)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    ctx.set_icp_variant(args.icp_variant)
    ctx.upload_scans(w.pts, w.offsets, params.downsample_icp_points_ratio)
    n_src = np.diff(w.offsets)[w.edges[:, 1]]
    n_tgt = np.diff(w.offsets)[w.edges[:, 0]]
    pl = D.plan(rank, world, w.E, w.n_successive, w.icp_factor_first, edge_cost=n_src * n_tgt, strategy=args.shard)
    e0, e1 = pl.edge_range
    ctx.icp_prepare(pl.edges(w.edges), w.est, params)
    F = pl.factors(w.factors_placeholder(), w.icp_factor_first)
    hb_size = ctx.gn_setup(w.V, F, pl.factor_range, gp)
    backend = D.DeviceBackend(ctx, hb_size, hb_size - 2, dev)
    X0 = w.est.astype(np.float64)

    def step():
        ctx.icp_run(compute_cov=True)
        ctx.gn_take_icp(w.icp_factor_first + e0, e1 - e0, pl.n_always_local, params)
        ctx.gn_set_poses(X0)
        return D.gn_loop(backend, lambda hb: dist.all_reduce(hb), gp)

    def barrier():
        torch.cuda.synchronize(dev)
        dist.barrier()
        torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        st = step()
    barrier()
    icp_ms, iters = [], []
    t_start = time.perf_counter()
    for _ in range(args.steps):
        st = step()
        torch.cuda.synchronize(dev)
        icp_ms.append(ctx.icp_kernel_ms())
        iters.append(st["iterations"])
    barrier()
    t = torch.tensor([time.perf_counter() - t_start, float(np.mean(icp_ms))], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, k_ms = float(t[0]), float(t[1])
    if rank == 0:
        print(json.dumps({
            "metric": "ICP edges/sec + ms/GN-iter on 5k-node/20k-edge synthetic graph, 1->8 GPU",
            "value": w.E * args.steps / elapsed, "unit": "edges/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "fp32 (ICP) + fp64 (GN)",
            "data": "synthetic (seeded ray-cast 2D world, 5000-beam scans -> ~1000-pt clouds)",
            "config": {"workload": f"{args.config}: {w.V} nodes / {w.E} ICP edges / {len(F)} factors",
                       "nodes": w.V, "icp_edges": w.E, "factors": len(F),
                       "parallelism": f"edge-sharded dp{world} (torch form)"},
            "form": "torch", "ranks": world, "icp_kernel_ms": k_ms, "gn_iterations": float(np.mean(iters)),
            "gn_loop": "python", "roofline": None, "cpu_baseline": None}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
