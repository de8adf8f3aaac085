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
    args = ap.parse_args()

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
