"""libdpg's one-process-per-GPU form at world > 1 on ONE card (run under torch.distributed.run,
gloo): dpg_ctx_create_rank_ops with dpgslam.dist.HostCollective as the collective -- RCCL refuses
two ranks on one device, so the rank form's three cross-process steps (the cost all-reduce of the
LPT plan, the results' all-gather in dpg_icp_batch_fetch, the all-reduce of the packed system per
Gauss-Newton iteration) run over gloo, and everything else is the code the RCCL rank form runs:
shard planning by global rank, factor ownership, the ICP-to-factor scatter, the vote words that keep
the ranks' stop decisions equal.  Every rank checks its results against a single-device context
(ICP results and covariance blocks byte-identical, the same GN iteration / factorization counts,
poses within 1e-9) under both dispatch schedules, and that the ranks issued the same collectives.
Prints "rank check ok" on every rank.
usage: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/rank_check.py [CONFIG]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpg-slam_amd"), os.path.join(ROOT, "tests")]


def main():
    import torch
    import torch.distributed as dist
    from dpgslam import _abi, api, synth
    from dpgslam import dist as D
    from multi_common import compare, run_all, run_step

    cfg = sys.argv[1] if len(sys.argv) > 1 else "config3"
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    torch.cuda.init()
    w = synth.generate(cfg)
    p = _abi.default_icp_params()
    small = cfg != "config4"

    def run(c):
        if small:
            out = run_all(c, w, p)
        else:
            c.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
            out = run_step(c, w, p)
        # pairs never aligned before (the edges reversed), run twice before any fetch: under the
        # measured schedule the second run plans from the first run's costs, all-reduced over ranks
        e2 = np.ascontiguousarray(w.edges[:, ::-1])
        c.icp_prepare(e2, w.est, p)
        c.icp_run(compute_cov=False)
        c.icp_run(compute_cov=False)
        r2, _ = c.icp_fetch(with_hessian=False)
        out["rev"] = r2.tobytes()
        return out

    coll = D.HostCollective()
    outs = {}
    for sched in ("caller", "measured"):
        with api.Context(0, rank_ops=(coll, rank, world)) as c:
            assert (c.n_gpus, c.n_ranks, c.rank) == (1, world, rank), (c.n_gpus, c.n_ranks, c.rank)
            c.set_icp_schedule(sched)
            outs[sched] = run(c)
        assert coll.error is None, coll.error
    with api.Context(0) as s:
        ref = run(s)
    for sched, out in outs.items():
        try:
            assert out["rev"] == ref["rev"], "reversed-pair batch differs"
            compare(out, ref)
        except AssertionError as e:
            raise AssertionError(f"rank {rank}, schedule {sched}: {e}") from None
    calls = [None] * world
    dist.all_gather_object(calls, dict(coll.calls))
    assert all(c == calls[0] for c in calls), calls
    assert coll.calls["allgather"] > 0 and coll.calls["allreduce_f64"] > 0 and coll.calls["allreduce_f32"] > 0, coll.calls
    dist.destroy_process_group()
    # the pipelined GN of the rank form over the host collective (its all-reduce on libdpg's
    # collective thread, no stream sync per iteration) beside the single-device loop; the two ranks
    # share ONE card, so this is a correctness run's clock, not a scaling number
    gn = {k: round(float(v["gnms1"]), 4) for k, v in (("rank_caller", outs["caller"]), ("rank_measured", outs["measured"]),
                                                   ("single", ref))}
    print(f"rank check ok: rank {rank} of {world}, {cfg}, collectives {coll.calls}, gn ms/iter {gn}", flush=True)


if __name__ == "__main__":
    main()
