"""Multi-rank path through libdpg (run under torch.distributed.run; every rank may share one GPU):
the bench step of bench.py -- edges sharded by cost (dpgslam.dist.plan), each rank's ICP batch,
its ICP factors, then Gauss-Newton with ONE all-reduce of the packed [H | g | chi2] buffer per
iteration (gloo here, RCCL with --backend nccl on separate GPUs) -- against the single-process
solve on rank 0: the shards' ICP results byte-identical to one batch over all edges, the poses
equal to dpg_optimize_graph's within 1e-9.  Prints "dist check ok".
usage: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/dist_check.py [CONFIG]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpg-slam_amd")]


def main():
    import torch
    import torch.distributed as dist
    from dpgslam import _abi, api, synth
    from dpgslam import dist as D

    cfg = sys.argv[1] if len(sys.argv) > 1 else "config3"
    backend = os.environ.get("DIST_BACKEND", "gloo")
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    gpu = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    dist.init_process_group(backend, device_id=dev) if backend == "nccl" else dist.init_process_group("gloo")
    w = synth.generate(cfg)
    p, gp = _abi.default_icp_params(), _abi.default_gn_params()
    ctx = api.Context(gpu)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
    n_src = np.diff(w.offsets)[w.edges[:, 1]]
    n_tgt = np.diff(w.offsets)[w.edges[:, 0]]
    pl = D.plan(rank, world, w.E, w.n_successive, w.icp_factor_first, edge_cost=n_src * n_tgt,
                strategy=os.environ.get("DIST_SHARD", "interleave"))
    e0, e1 = pl.edge_range
    ctx.icp_prepare(pl.edges(w.edges), w.est, p)
    F = pl.factors(w.factors_placeholder(), w.icp_factor_first)
    hb_size = ctx.gn_setup(w.V, F, pl.factor_range, gp)
    be = D.DeviceBackend(ctx, hb_size, hb_size - 2, dev)
    ctx.icp_run(compute_cov=False)
    ctx.gn_take_icp(w.icp_factor_first + e0, e1 - e0, pl.n_always_local, p)
    ctx.gn_set_poses(w.est.astype(np.float64))
    st = D.gn_loop(be, (lambda hb: dist.all_reduce(hb)), gp)
    torch.cuda.synchronize(dev)
    X = ctx.gn_get_poses(w.V)
    res, _ = ctx.icp_fetch(with_hessian=False)
    parts = [None] * world
    dist.all_gather_object(parts, (e0, e1, res.tobytes(), X.tobytes()))
    if rank == 0:
        ref_res, _ = ctx.icp_batch(w.edges, w.est, p, compute_cov=False)
        for a, b, rb, xb in parts:
            mine = ref_res[pl.perm[a:b]].tobytes()   # the same edges of one batch over all
            assert rb == mine, f"ICP results of shard [{a}, {b}) differ from one batch"
            assert xb == parts[0][3], "ranks disagree on the poses"
        Xr, st_r = ctx.optimize_graph(w.est.astype(np.float64), w.factors_with_icp(ref_res, p))
        d = float(np.abs(X - Xr).max())
        print(f"{cfg}: world {world}, edges per rank {[b - a for a, b, _, _ in parts]}, GN iterations "
              f"{st['iterations']} (single process {st_r.iterations}), max |pose difference| {d:.3e}", flush=True)
        assert d < 1e-9, d
        print("dist check ok", flush=True)
    dist.barrier()
    dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
