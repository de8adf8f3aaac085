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
    prof, pbuf = [], (C.c_double * 8)()
    lat, icp_ms, sym_ms, num_ms, reord, relin = [], [], [], [], 0, 0
    with api.Context(0) as ctx:
        g = api.IncGraph(ctx, mode=args.inc_mode)
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
            L.dpg_inc_last_profile(C.c_void_p(g.handle), pbuf, 8)
            prof.append(list(pbuf)[:6])
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
                                                          "chol_host", "chol_upload"],
                                                         np.mean(np.asarray(prof[-500:]), 0).round(4).tolist()))},
        "reorders": reord, "relinearized_total": relin, "nnz_L_blocks": nnz, "factors": n_fac,
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
    ap.add_argument("--workload", default="batch", choices=["batch", "incremental"],
                    help="batch: the headline step (all edges + GN); incremental: per-node latency of "
                         "dpg_add_node_pairs at V = 5000 (1 GPU)")
    ap.add_argument("--inc-mode", default="isam2", choices=["isam2", "batch"])
    ap.add_argument("--inc-nodes", type=int, default=5000)
    ap.add_argument("--cpu-nodes", type=int, default=8, help="nodes in the incremental CPU-baseline sample")
    args = ap.parse_args()
    if args.workload == "incremental":
        return main_incremental(args)

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE")

    import torch
    import torch.distributed as dist
    from dpgslam import _abi, api, synth
    from dpgslam import dist as D

    gpu = local_rank % max(1, torch.cuda.device_count())   # == local_rank on a full node
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)   # RCCL over xGMI
        else:
            dist.init_process_group("gloo")

    t0 = time.time()
    w = synth.generate(args.config)
    log(f"[rank {rank}] generated {args.config}: V={w.V} E={w.E} points={len(w.pts)} in {time.time() - t0:.1f}s")
    params = _abi.default_icp_params()
    gp = _abi.default_gn_params()

    ctx = api.Context(gpu)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    ctx.set_icp_variant(args.icp_variant)
    ctx.upload_scans(w.pts, w.offsets, params.downsample_icp_points_ratio)
    n_src = np.diff(w.offsets)[w.edges[:, 1]]
    n_tgt = np.diff(w.offsets)[w.edges[:, 0]]
    pl = D.plan(rank, world, w.E, w.n_successive, w.icp_factor_first, edge_cost=n_src * n_tgt)
    e0, e1 = pl.edge_range
    my_edges = w.edges[e0:e1]
    ctx.icp_prepare(my_edges, w.est, params)
    F = w.factors_placeholder()
    hb_size = ctx.gn_setup(w.V, F, pl.factor_range, gp)
    backend = D.DeviceBackend(ctx, hb_size, hb_size - 2, dev)
    allreduce = (lambda hb: dist.all_reduce(hb)) if world > 1 else (lambda hb: None)
    X0 = w.est.astype(np.float64)

    def step():
        ctx.icp_run(compute_cov=True)
        ctx.gn_take_icp(w.icp_factor_first + e0, e1 - e0, pl.n_always_local, params)
        ctx.gn_set_poses(X0)
        return D.gn_loop(backend, allreduce, gp)

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        st = step()
    barrier()
    icp_ms, cov_ms, idx_ms, gn_iters, gn_ms, n_fact = [], [], [], [], [], []
    t_start = time.perf_counter()
    for _ in range(args.steps):
        ts = time.perf_counter()
        st = step()
        torch.cuda.synchronize(dev)
        icp_ms.append(ctx.icp_kernel_ms())
        cov_ms.append(ctx.cov_kernel_ms())
        idx_ms.append(ctx.kdtree_build_ms())
        gn_iters.append(st["iterations"])
        n_fact.append(ctx.gn_factorizations())
        gn_ms.append((time.perf_counter() - ts) * 1e3 - icp_ms[-1] - cov_ms[-1] - idx_ms[-1])
    barrier()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_step = elapsed * 1e3 / args.steps
    algo_bytes = ctx.icp_algorithmic_bytes()
    k_ms = float(np.mean(icp_ms))
    achieved = algo_bytes / (k_ms * 1e-3) / 1e9
    res, _ = ctx.icp_fetch(with_hessian=False)
    stats = {"icp_kernel_ms": k_ms, "cov_kernel_ms": float(np.mean(cov_ms)), "index_build_ms": float(np.mean(idx_ms)), "gn_iterations": float(np.mean(gn_iters)), "gn_factorizations": float(np.mean(n_fact)),
             "ms_per_gn_iter": float(np.mean(gn_ms) / max(1.0, np.mean(gn_iters))),
             "icp_iters_mean": float(res["iterations"].mean()), "icp_iters_max": int(res["iterations"].max()),
             "final_error": st["final_error"], "pcg_iterations": st["pcg_iterations"]}
    if world > 1:
        t = torch.tensor([stats["icp_kernel_ms"], stats["ms_per_gn_iter"]], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        stats["icp_kernel_ms"], stats["ms_per_gn_iter"] = float(t[0]), float(t[1])

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
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
        # the same ICP sample over edges with OpenMP, at most 16 threads (the box's share)
        nt = max(1, min(16, cores.get("affinity") or 1))
        if nt > 1:
            cm = cpu_baseline(w, params, args.cpu_sample, threads=nt)
            cpu["multithread"] = {"value": cm["icp_edges_per_s"], "unit": "edges/s", "cores": nt,
                                  "sample": f"same sample, OpenMP over edges, median of 5 runs ({cm['icp_s']:.2f} s per run)"}

    traffic, traffic_src, sq = pmc_traffic(KERNEL_NAME[args.icp_variant])
    if world > 1:   # the PMC pass measured the whole 1-GPU launch; a rank's launch holds only its shard
        traffic, traffic_src, sq = None, None, {}
    if rank == 0:
        line = {
            "metric": "ICP edges/sec + ms/GN-iter on 5k-node/20k-edge synthetic graph, 1->8 GPU",
            "value": w.E * args.steps / elapsed,
            "unit": "edges/s",
            "n_gpus": world,
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
                       "nodes": w.V, "icp_edges": w.E, "factors": len(F), "parallelism": f"edge-sharded dp{world}"},
            "ms_per_gn_iter": stats["ms_per_gn_iter"],
            "gn_iterations": stats["gn_iterations"],
            "gn_factorizations": stats["gn_factorizations"],
            "icp_kernel_ms": stats["icp_kernel_ms"],
            "cov_kernel_ms": stats["cov_kernel_ms"],
            "index_build_ms": stats["index_build_ms"],
            "icp_variant": args.icp_variant,
            "icp_edges_per_s_kernel": w.E / world / (stats["icp_kernel_ms"] * 1e-3) * world,
            "icp_iters_mean": stats["icp_iters_mean"],
            "icp_iters_max": stats["icp_iters_max"],
            "gn_note": "ms_per_gn_iter averages plain GN steps and chord steps that reuse the last Cholesky "
                       "factor (gn_factorizations of gn_iterations refactor; DESIGN.md section 3)",
            # roofline of the dominant kernel against HBM (SURVEY 8d's algorithmic bytes); the counters
            # say what actually limits it: "limiter" + the SQ fractions of the last committed PMC pass
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": KERNEL_NAME[args.icp_variant] + " (correspondence search + fit, fused)",
                         "bytes_per_launch": algo_bytes,
                         "limiter": "VALU issue + LDS latency with per-iteration workgroup barriers, not HBM: "
                                    "the clouds stay in LDS for all iterations (traffic << algorithmic bytes)",
                         **({"sq": sq} if sq else {})},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
