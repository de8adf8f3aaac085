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
    """HBM bytes per launch of `kernel` from the last committed rocprofv3 PMC pass
    (profiles/pmc_traffic.json, written by tools/pmc_summary.py: (2 x FETCH_SIZE + WRITE_SIZE) KiB,
    the gfx950 correction of MI355X_MICROARCH.md "HBM").  None when no pass covers this kernel."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None, None
    d = json.load(open(path))
    for k, v in d.get("traffic_bytes_per_launch", {}).items():
        if k.split("<")[0] == kernel:
            return float(v), d.get("source")
    return None, None


def cpu_baseline(w, params, sample_edges: int, threads: int = 1) -> dict:
    """Oracle (CPU restatement, grid NN) timed on this host: ICP on a bounded sample of the same
    workload + the full-graph GN (block-sparse Cholesky)."""
    from oracle import oracle as O
    rng = np.random.default_rng(0)
    sel = np.sort(rng.choice(w.E, min(sample_edges, w.E), replace=False))
    O.icp_batch(w.pts, w.offsets, w.edges[sel[:8]], w.est, params, O.NN_GRID, threads)   # warm-up
    t0 = time.perf_counter()
    res, _ = O.icp_batch(w.pts, w.offsets, w.edges[sel], w.est, params, O.NN_GRID, threads)
    t_icp = time.perf_counter() - t0
    # GN on the full graph needs all ICP measurements: use the GPU's (bit-identical) results
    return {"icp_edges_per_s": len(sel) / t_icp, "icp_s": t_icp, "n": len(sel), "iters_mean": float(res["iterations"].mean())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="config4")
    ap.add_argument("--cpu-sample", type=int, default=1500, help="edges in the CPU-baseline sample")
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
        cb = cpu_baseline(w, params, args.cpu_sample, threads=1)
        cpu = {"value": cb["icp_edges_per_s"], "unit": "edges/s", "cores": 1, "kind": "port",
               "sample": f"oracle (C restatement, grid NN, 1 thread) ICP on {cb['n']} random edges of "
                         f"{args.config} ({cb['icp_s']:.1f} s, mean {cb['iters_mean']:.1f} ICP iterations)"}
        # the same sample over edges with OpenMP, at most 16 threads (the box's share)
        nt = max(1, min(16, os.cpu_count() or 1))
        if nt > 1:
            cm = cpu_baseline(w, params, args.cpu_sample, threads=nt)
            cpu["multithread"] = {"value": cm["icp_edges_per_s"], "unit": "edges/s", "cores": nt,
                                  "sample": f"same sample, OpenMP over edges ({cm['icp_s']:.2f} s)"}

    traffic, traffic_src = pmc_traffic(KERNEL_NAME[args.icp_variant])
    if world > 1:   # the PMC pass measured the whole 1-GPU launch; a rank's launch holds only its shard
        traffic, traffic_src = None, None
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
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": KERNEL_NAME[args.icp_variant] + " (correspondence search + fit, fused)",
                         "bytes_per_launch": algo_bytes},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
