"""The C-ABI library loads on any host and exports every function include/*.h declares; the
host-side data path (R1-R3, R9) is bit-identical to the oracle's restatement.  No GPU calls."""
import ctypes as C
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_functions():
    names = set()
    for h in ("dpg_slam_c.h", "dpg_icp_cov.h"):
        txt = open(os.path.join(ROOT, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b(\w+)\s*\(", txt, flags=re.M):
            if m.group(1) not in ("if", "defined"):
                names.add(m.group(1))
    return sorted(names)


def test_library_exports_every_declared_symbol():
    from dpgslam import _abi
    L = C.CDLL(_abi.LIB_PATH)
    names = _declared_functions()
    assert len(names) >= 35
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert set(names) == set(_abi.SIGNATURES), set(names) ^ set(_abi.SIGNATURES)


def _c_layout(struct, fields):
    """sizeof and field offsets of a header struct, as gcc lays it out."""
    import subprocess
    import tempfile
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    body = "".join(f'printf(" %zu", offsetof({struct}, {f}));' for f in fields)
    src = (f'#include <stddef.h>\n#include <stdio.h>\n#include "dpg_slam_c.h"\n'
           f'int main(void) {{ printf("%zu", sizeof({struct})); {body} return 0; }}\n')
    with tempfile.TemporaryDirectory() as d:
        open(os.path.join(d, "l.c"), "w").write(src)
        subprocess.run(["gcc", "-I", inc, "-o", os.path.join(d, "l"), os.path.join(d, "l.c")], check=True)
        out = subprocess.run([os.path.join(d, "l")], check=True, capture_output=True, text=True).stdout.split()
    return [int(x) for x in out]


def test_struct_layouts():
    from dpgslam import _abi
    assert C.sizeof(_abi.IcpResult) == 64 and C.sizeof(_abi.Factor) == 64
    for struct, cls in (("dpg_icp_params", _abi.IcpParams), ("dpg_gn_params", _abi.GnParams),
                        ("dpg_gn_stats", _abi.GnStats), ("dpg_change_params", _abi.ChangeParams),
                        ("dpg_change_stats", _abi.ChangeStats)):
        names = [f[0] for f in cls._fields_]
        lay = _c_layout(struct, names)
        assert lay[0] == C.sizeof(cls), (struct, lay[0], C.sizeof(cls))
        assert lay[1:] == [getattr(cls, n).offset for n in names], (struct, lay[1:])
    p = _abi.default_icp_params()
    assert (p.icp_maximum_iterations, p.icp_use_reciprocal_correspondences, p.downsample_icp_points_ratio) == (500, 1, 5)
    assert p.icp_maximum_transformation_epsilon == 0.000000005 and p.icp_max_correspondence_distance == 0.6
    assert (p.laser_x_variance, p.laser_y_variance) == (0.5, 0.5) and p.laser_theta_variance == np.float32(0.3)


def test_no_gpu_means_loud_failure():
    """Without a HIP device the product path fails loudly (no CPU fallback)."""
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is present")
    from dpgslam import api, _abi
    with pytest.raises(_abi.DpgError):
        api.Context(0)


def test_host_data_path_matches_oracle(workload):
    """R1 scan->cloud, R2 downsample, R3 guess / transforms: product host code == oracle, bitwise."""
    from dpgslam import api, synth
    from oracle import oracle as O
    w = workload("config1")
    for v in range(2):
        a = api.scan_to_cloud(w.ranges[v], synth.ANGLE_MIN, synth.ANGLE_MAX, synth.RANGE_MAX)
        b = O.scan_to_cloud(w.ranges[v], synth.ANGLE_MIN, synth.ANGLE_MAX, synth.RANGE_MAX)
        assert a.tobytes() == b.tobytes() == w.cloud(v).tobytes()
        for r in (1, 3, 5):
            assert api.downsample(a, r).tobytes() == O.downsample(a, r).tobytes()
    rng = np.random.default_rng(1)
    for _ in range(200):
        p, q = rng.normal(0, 10, 3).astype(np.float32), rng.normal(0, 10, 3).astype(np.float32)
        assert api.inverse_transform_point(p, q).tobytes() == O.inverse_transform_point(p, q).tobytes()
        assert api.transform_point(p, q).tobytes() == O.transform_point(p, q).tobytes()
        assert api.icp_guess(p, q).tobytes() == O.icp_guess(p, q).tobytes()
    # MAX_RANGE beams are dropped (dpg_measurement.h:43: range >= max_range)
    r = np.array([1.0, 30.0, 31.0, 2.0], np.float32)
    assert len(api.scan_to_cloud(r, -1.0, 1.0, 30.0)) == 2
    assert len(api.scan_to_cloud(np.zeros(0, np.float32), -1.0, 1.0, 30.0)) == 0


def test_odometry_factor_noise_model():
    """dpg_slam.cc:56-75: sigma_t = 0.4*|d| + 0.4*|dtheta| (float), Diagonal::Sigmas."""
    from dpgslam import api
    f = api.odometry_factor([0, 0, 0], [1.0, 0.0, 0.1], 3, 4)
    st = np.float32(0.4) * np.float32(1.0) + np.float32(0.4) * np.float32(0.1)
    assert (f.i, f.j) == (3, 4)
    assert f.info[0] == 1.0 / (float(st) * float(st)) and f.info[2] == f.info[0]
    assert abs(f.z[2] - 0.1) < 1e-7


def test_batched_factor_builders_equal_per_factor_calls():
    """reoptimize builds its prior / odometry factors for all nodes at once (dpg_odometry_factors,
    api.prior_factors): byte-identical to the per-node calls of the reference's loop
    (dpg_slam.cc:41-75), in node order; a zero-motion pair fails the batch as it fails the single call."""
    from dpgslam import _abi, api
    from dpgslam._abi import FACTOR_DTYPE
    rng = np.random.default_rng(7)
    odom = np.cumsum(rng.normal(0, 0.3, (50, 3)), 0).astype(np.float32)
    a = np.arange(0, 49, dtype=np.int32)
    b = a + 1
    motion = (0.4, 0.3, 0.2, 0.1)
    Fb = api.odometry_factors(odom, a, b, motion)
    for k in range(len(a)):
        f = np.frombuffer(bytes(api.odometry_factor(odom[a[k]], odom[b[k]], int(a[k]), int(b[k]), motion)), FACTOR_DTYPE)
        assert Fb[k].tobytes() == f.tobytes(), k
    Pb = api.prior_factors([0, 7, 30], sigmas=(0.2, 0.25, 0.15))
    for k, n in enumerate([0, 7, 30]):
        assert Pb[k].tobytes() == api.prior_factor(n, sigmas=(0.2, 0.25, 0.15)).tobytes()
    with pytest.raises(_abi.DpgError):
        api.odometry_factors(np.zeros((2, 3), np.float32), [0], [1], motion)
