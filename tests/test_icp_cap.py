"""The ICP iteration cap and the reciprocal test's drift bound (DESIGN.md K1 "drift").

The reciprocal test searches the STATIC source index with a window widened by 1e-4 + 5e-5 (k + 1) m
for the float drift of the incrementally moved source points (dpg_icp_ang.hip, dpg_icp_kd.hip);
the bound is loosest where the drift is largest, after many iterations.  Here transformation
epsilon 0 and MSE threshold 0 (PCL's convergence criteria can then only fire on an exact identity
step) drive config-2 edges to the 500-iteration cap (icp_maximum_iterations, dpg_slam.cc:412),
and the outcome must stay bit-exact against the oracle.  The diagnostics build
(lib/libdpg_stats.so) measures the drift itself: the largest |moved - (F p + t)| over every moved
point must stay below the margin the next reciprocal test adds for it, on config 4 and on the
capped edges."""
import os
import re
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _capped():
    from dpgslam import _abi
    p = _abi.default_icp_params()
    p.icp_maximum_transformation_epsilon = 0.0
    p.mse_threshold_absolute = 0.0
    return p


@pytest.mark.parametrize("variant", ["angular", "kdtree"])
def test_icp_iteration_cap_bit_exact(ctx, workload, variant):
    from oracle import oracle as O
    w = workload("config2")
    p = _capped()
    edges = w.edges[::20][:25]
    ctx.set_icp_variant(variant)
    ctx.upload_scans(w.pts, w.offsets, 5)
    res, _ = ctx.icp_batch(edges, w.est, p, compute_cov=False)
    ctx.set_icp_variant("angular")
    ref, _ = O.icp_batch(w.pts, w.offsets, edges, w.est, p, O.NN_GRID, threads=16)
    for k in ("T", "z", "converged", "iterations", "n_corr", "status", "fitness"):
        assert np.array_equal(np.asarray(res[k]), np.asarray(ref[k])), k
    assert (res["iterations"] == p.icp_maximum_iterations).mean() >= 0.5, res["iterations"]


def _drift_ratio(args):
    lib = os.path.join(ROOT, "dpg-slam_amd", "lib", "libdpg_stats.so")
    if not os.path.exists(lib):
        pytest.fail("lib/libdpg_stats.so is missing: build it with `make -C dpg-slam_amd stats` (__graft_entry__.build)")
    env = dict(os.environ, DPGSLAM_LIB=lib)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "icp_stats.py")] + args, env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    m = re.search(r"max \|moved - F p\| ([0-9.e+-]+) m, max drift / window margin ([0-9.e+-]+)", out.stdout)
    assert m, out.stdout
    return float(m.group(1)), float(m.group(2))


@pytest.mark.parametrize("args", [["config4"], ["config2", "--cap", "--edges", "60"]], ids=["config4", "config2-cap"])
def test_reciprocal_drift_within_margin(args):
    drift, ratio = _drift_ratio(args)
    print(f"{' '.join(args)}: max drift {drift:.3e} m, {ratio:.4f} of the margin")
    assert 0.0 < ratio < 1.0
