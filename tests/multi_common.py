"""Shared by the multi-device tests (tests/test_multi_gpu_ctx.py) and the two-process rank-form
check (tools/rank_check.py): one run of every sharded entry point on a context, and the pose error."""
import numpy as np

from conftest import angle_wrap


def perr(A, B):
    return float(np.abs(np.concatenate([A[:, :2] - B[:, :2], angle_wrap(A[:, 2:] - B[:, 2:])], 1)).max())


def run_all(ctx, w, p, sweep=True):
    """ICP batch (+ covariance) twice (the second run re-plans from the first run's costs), the
    graph solve, the bench's step form, and a sweep."""
    from dpgslam import _abi
    ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
    res1, hess1 = ctx.icp_batch(w.edges, w.est, p, compute_cov=True)
    ctx.icp_run(compute_cov=True)           # again: the measured schedule now (LPT + longest first)
    res2, hess2 = ctx.icp_fetch(with_hessian=True)
    F = w.factors_with_icp(res1, p)
    X, st = ctx.optimize_graph(w.est.astype(np.float64), F)
    out = dict(res1=res1.tobytes(), hess1=np.asarray(hess1).tobytes(), res2=res2.tobytes(),
               hess2=np.asarray(hess2).tobytes(), X=X, it=st.iterations)
    out.update(run_step(ctx, w, p))
    if sweep:
        passes = np.zeros(w.V, np.int32)
        passes[w.V // 2:] = 1
        Xr, sr = ctx.reoptimize(passes, w.est, w.odom)
        rr, _ = ctx.icp_fetch(with_hessian=False)
        out.update(Xr=Xr, itr=sr.gn.iterations, nlc=sr.n_loop_closures, rr=rr.tobytes())
    return out


def run_step(ctx, w, p):
    """bench.py's step: the staged batch's results become factors on the device(s) that aligned
    them, then the Gauss-Newton loop (run twice: the second on the measured schedule)."""
    from dpgslam import _abi
    out = {}
    for k in range(2):
        ctx.icp_prepare(w.edges, w.est, p)
        ctx.icp_run(compute_cov=True)
        rs, hs = ctx.icp_fetch(with_hessian=True)
        gp = _abi.default_gn_params()
        ctx.gn_setup(w.V, w.factors_placeholder(), params=gp)
        ctx.gn_take_icp(w.icp_factor_first, w.E, w.n_successive, p)
        ctx.gn_set_poses(w.est.astype(np.float64))
        sst, Xs = ctx.gn_run(w.V)
        out.update({f"rs{k}": rs.tobytes(), f"hs{k}": np.asarray(hs).tobytes(), f"Xs{k}": Xs,
                    f"its{k}": sst["iterations"], f"nfs{k}": ctx.gn_factorizations(), f"err_s{k}": sst["final_error"],
                    f"gnms{k}": sst["ms_per_iteration"]})
    return out


BYTE_KEYS = ("res1", "hess1", "res2", "hess2", "rs0", "hs0", "rs1", "hs1", "rr")


def compare(out, ref, exact_poses=False):
    """The multi-device bar: ICP results and covariance blocks byte-identical, the same GN
    iteration / factorization counts, poses within 1e-9 (bitwise with exact_poses)."""
    for key in BYTE_KEYS:
        if key in ref:
            assert out[key] == ref[key], f"{key} differs from the single-device context"
    pose_keys = [(x, i) for x, i in (("X", "it"), ("Xs0", "its0"), ("Xs1", "its1"), ("Xr", "itr")) if x in ref]
    for xk, ik in pose_keys:
        assert out[ik] == ref[ik], (ik, out[ik], ref[ik])
        if exact_poses:
            assert out[xk].tobytes() == ref[xk].tobytes(), xk
        else:
            assert perr(out[xk], ref[xk]) < 1e-9, (xk, perr(out[xk], ref[xk]))
    for k in ("nfs0", "nfs1"):
        assert out[k] == ref[k], (k, out[k], ref[k])
    for k in ("err_s0", "err_s1"):
        assert abs(out[k] - ref[k]) <= 1e-9 * max(1.0, abs(ref[k])), (k, out[k], ref[k])
    if "nlc" in ref:
        assert out["nlc"] == ref["nlc"]
