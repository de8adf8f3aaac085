#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ (data only).

  config1_golden.npz  config 1 (two 360-beam scans, seed 1): the oracle's complete runIcp outcome
                      at downsample ratio 5 and 1 (clouds, guess, per-iteration correspondence
                      indices, final transform, measurement, flags, covariance + Hessian block)
  cov_expr.npz        the reference's OWN generated expressions for d2J_da2, d2J_dxda, d2J_dyda
                      (src/icp_cov/cov_func_point_to_point.h:133-165), evaluated in float64 at
                      seeded random inputs with b = c = 0 (T20 = T21 = 0, T22 = 1) and z = 0.
                      Needs /root/reference (read as text, evaluated as arithmetic); the inputs
                      and outputs are stored so the tests never read the reference.
  cov6_expr.npz       the same for ALL 36 d2J_dX2 entries and all 36 d2J_dZdX entries of one
                      point (:45-281, :311-528), in the reference's row/column layout, and the
                      commented-out 6x6 sandwich (:553-566) over seeded clouds: d2J_dX2 summed
                      over every index pair, d2J_dZdX over the first min(n, 200), cov_z = 0.01 I,
                      bigger = inv(H) B cov_z B^T inv(H) and its [x, y, yaw] block (:563-566).

Run from the repo root:  PYTHONPATH=.:dpg-slam_amd python tests/golden/make_golden.py
"""
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpg-slam_amd")]
REF_COV = "/root/reference/src/icp_cov/cov_func_point_to_point.h"


def make_config1():
    from dpgslam import _abi, api, synth
    from oracle import oracle as O
    w = synth.generate("config1")
    out = {"ranges": w.ranges, "est": w.est, "angle_min": synth.ANGLE_MIN, "angle_max": synth.ANGLE_MAX,
           "range_max": synth.RANGE_MAX, "cloud0": w.cloud(0), "cloud1": w.cloud(1)}
    for ratio in (5, 1):
        p = _abi.default_icp_params()
        p.downsample_icp_points_ratio = ratio
        sd, td = api.downsample(w.cloud(1), ratio), api.downsample(w.cloud(0), ratio)
        g = O.icp_guess(w.est[1], w.est[0])
        res, tr = O.icp_align(sd, td, g, p, O.NN_BRUTE, trace_iters=100)
        cov, hess = O.icp_cov(w.cloud(1), w.cloud(0), np.array(res.T, np.float32))
        r = np.frombuffer(bytes(res), _abi.RESULT_DTYPE)
        out.update({f"r{ratio}_guess": g, f"r{ratio}_trace": tr[:res.iterations], f"r{ratio}_result": r,
                    f"r{ratio}_cov": cov, f"r{ratio}_hess": hess})
    np.savez_compressed(os.path.join(HERE, "config1_golden.npz"), **out)
    print("config1_golden.npz written")


def _expr(src: str, name: str) -> str:
    m = re.search(rf"\b{name}\s*=\s*(.*?);", src, flags=re.S)
    if not m:
        raise RuntimeError(f"{name} not found")
    return " ".join(m.group(1).split())


def make_cov_expr():
    if not os.path.exists(REF_COV):
        print("reference not mounted; cov_expr.npz kept as is")
        return
    src = open(REF_COV).read()
    exprs = {k: _expr(src, k) for k in ("d2J_da2", "d2J_dxda", "d2J_dyda")}
    rng = np.random.default_rng(20201127)
    n = 400
    inp = {"a": rng.uniform(-np.pi, np.pi, n), "x": rng.normal(0, 2, n), "y": rng.normal(0, 2, n),
           "pix": rng.normal(0, 10, n), "piy": rng.normal(0, 10, n), "qix": rng.normal(0, 10, n),
           "qiy": rng.normal(0, 10, n)}
    env = dict(inp, b=np.zeros(n), c=np.zeros(n), z=np.zeros(n), piz=np.zeros(n), qiz=np.zeros(n),
               sin=np.sin, cos=np.cos, pow=np.power)
    out = dict(inp)
    for k, e in exprs.items():
        out[k] = np.asarray(eval(e, {"__builtins__": {}}, env), np.float64)   # arithmetic only
    np.savez_compressed(os.path.join(HERE, "cov_expr.npz"), **out)
    print("cov_expr.npz written")


X_NAMES = ["x", "y", "z", "a", "b", "c"]
Z_NAMES = ["pix", "piy", "piz", "qix", "qiy", "qiz"]


def _h_name(i, j):
    """The reference's variable in row i, column j of d2J_dX2_temp (:271-279)."""
    if i == j:
        return f"d2J_d{X_NAMES[i]}2"
    return f"d2J_d{X_NAMES[j]}d{X_NAMES[i]}"


def make_cov6():
    if not os.path.exists(REF_COV):
        print("reference not mounted; cov6_expr.npz kept as is")
        return
    src = open(REF_COV).read()
    hx = {(i, j): _expr(src, _h_name(i, j)) for i in range(6) for j in range(6)}
    bx = {(i, j): _expr(src, f"d2J_d{Z_NAMES[j]}_d{X_NAMES[i]}") for i in range(6) for j in range(6)}

    def ev(e, env):
        return np.asarray(eval(e, {"__builtins__": {}}, env), np.float64)   # arithmetic only

    def blocks(pts_p, pts_q, a, x, y):
        n = len(pts_p)
        env = {"a": np.full(n, a), "x": np.full(n, x), "y": np.full(n, y), "b": np.zeros(n), "c": np.zeros(n),
               "z": np.zeros(n), "pix": pts_p[:, 0], "piy": pts_p[:, 1], "piz": np.zeros(n), "qix": pts_q[:, 0],
               "qiy": pts_q[:, 1], "qiz": np.zeros(n), "sin": np.sin, "cos": np.cos, "pow": np.power}
        H = np.zeros((n, 6, 6))
        B = np.zeros((n, 6, 6))
        for (i, j), e in hx.items():
            H[:, i, j] = ev(e, env)
        for (i, j), e in bx.items():
            B[:, i, j] = ev(e, env)
        return H, B

    rng = np.random.default_rng(20260315)
    out = {}
    # per point, 400 random inputs
    n = 400
    a = rng.uniform(-np.pi, np.pi, n)
    x, y = rng.normal(0, 2, n), rng.normal(0, 2, n)
    P, Q = rng.normal(0, 10, (n, 2)), rng.normal(0, 10, (n, 2))
    Hs, Bs = np.zeros((n, 6, 6)), np.zeros((n, 6, 6))
    for k in range(n):
        h, bb = blocks(P[k:k + 1], Q[k:k + 1], a[k], x[k], y[k])
        Hs[k], Bs[k] = h[0], bb[0]
    out.update({"pt_a": a, "pt_x": x, "pt_y": y, "pt_p": P, "pt_q": Q, "pt_H": Hs, "pt_B": Bs})
    # sandwiches: float clouds as calculate_ICP_COV receives them, a planar float transform
    for c, (nd, nm) in enumerate([(300, 280), (150, 150), (1000, 1200)]):
        p = rng.normal(0, 8, (nd, 2)).astype(np.float32)
        q = (p[:nm] if nm <= nd else np.concatenate([p, rng.normal(0, 8, (nm - nd, 2)).astype(np.float32)]))
        q = (q + rng.normal(0, 0.05, q.shape)).astype(np.float32)
        th = np.float32(rng.uniform(-0.5, 0.5))
        T = np.eye(4, dtype=np.float32)
        T[0, 0], T[0, 1], T[1, 0], T[1, 1] = np.cos(th), -np.sin(th), np.sin(th), np.cos(th)
        T[0, 3], T[1, 3] = np.float32(rng.normal(0, 0.3)), np.float32(rng.normal(0, 0.3))
        yaw = float(np.arctan2(T[1, 0], T[0, 0]).astype(np.float32))   # atan2f; the oracle restates it exactly
        nh, nb = min(nd, nm), min(nd, nm, 200)
        h, _ = blocks(p[:nh].astype(np.float64), q[:nh].astype(np.float64), yaw, float(T[0, 3]), float(T[1, 3]))
        _, bb = blocks(p[:nb].astype(np.float64), q[:nb].astype(np.float64), yaw, float(T[0, 3]), float(T[1, 3]))
        H = h.sum(0)
        Bm = np.concatenate(list(bb), axis=1)   # 6 x 6 nb, block k = point k
        Hi = np.linalg.inv(H)
        big = Hi @ Bm @ (0.01 * np.eye(6 * nb)) @ Bm.T @ Hi
        out.update({f"s{c}_p": p, f"s{c}_q": q, f"s{c}_T": T, f"s{c}_yaw": np.float64(yaw), f"s{c}_H": H,
                    f"s{c}_M": Bm @ Bm.T, f"s{c}_cov6": big, f"s{c}_cov3": big[np.ix_([0, 1, 3], [0, 1, 3])]})
    np.savez_compressed(os.path.join(HERE, "cov6_expr.npz"), **out)
    print("cov6_expr.npz written")


if __name__ == "__main__":
    make_config1()
    make_cov_expr()
    make_cov6()
