"""GN solve policy A/B on config 4 (GPU box): the ICP measurements of one batched ICP, then the batch
Gauss-Newton (dpg_optimize_graph) under several refactor_delta values (chord steps reuse the
Cholesky factor once max|delta| < refactor_delta) -- iterations, factorizations, ms per iteration
and the largest pose difference to the oracle's plain Gauss-Newton on the same measurements.
usage: python tools/gn_policy.py [deltas...]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpg-slam_amd")]
import numpy as np  # noqa: E402

from dpgslam import _abi, api, synth  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    deltas = [float(x) for x in sys.argv[1:]] or [1e-4, 1e-3, 1e-2, 1e-1, 1.0]
    w = synth.generate("config4")
    p = _abi.default_icp_params()
    ctx = api.Context(0)
    ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
    res, _ = ctx.icp_batch(w.edges, w.est, p, compute_cov=False)
    F = w.factors_with_icp(res, p)
    X0 = w.est.astype(np.float64)
    t = time.time()
    Xo, sto = O.optimize_graph(X0, F)
    print(f"oracle GN: {sto.iterations} iterations, {time.time() - t:.2f} s", file=sys.stderr, flush=True)
    for d in deltas:
        gp = _abi.default_gn_params()
        gp.refactor_delta = d
        ctx.optimize_graph(X0, F, gp)   # warm-up (symbolic analysis cached per pattern? no: timed below per call)
        ms, its = [], []
        for _ in range(5):
            X, st = ctx.optimize_graph(X0, F, gp)
            ms.append(st.ms_per_iteration)
            its.append(st.iterations)
        print(json.dumps({"refactor_delta": d, "iterations": its[-1], "ms_per_iteration": float(np.median(ms)),
                          "ms_loop": float(np.median(ms)) * its[-1], "max_pose_diff_vs_oracle": float(np.abs(X - Xo).max()),
                          "final_error": st.final_error, "oracle_final_error": sto.final_error}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
