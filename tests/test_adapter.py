"""include/dpg_slam_adapter.hpp: the reference's entry points (calculate_ICP_COV
cov_func_point_to_point.h:24, DpgSLAM::runIcp dpg_slam.h:630, optimizeGraph dpg_slam.h:464,
reoptimize, executeDPG) over the C ABI, exercised by tools/adapter_check.cpp with stand-ins for
PCL / Eigen / DpgNode / PoseGraphParameters.  CPU: it compiles warning-free and links against
lib/libdpg.so.  GPU: every adapter call equals the direct C-ABI call bit for bit."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "dpg-slam_amd", "lib")


def test_adapter_compiles_and_links(tmp_path):
    out = str(tmp_path / "adapter_check")
    r = subprocess.run(["g++", "-O1", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-I" + os.path.join(ROOT, "include"),
                        "-o", out, os.path.join(ROOT, "tools", "adapter_check.cpp"), "-L" + LIBDIR, "-ldpg"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@pytest.mark.gpu
def test_adapter_matches_c_abi():
    exe = os.path.join(LIBDIR, "adapter_check")
    assert os.path.exists(exe), "build it with `make -C dpg-slam_amd adapter` (__graft_entry__.build)"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=dict(os.environ, LD_LIBRARY_PATH=LIBDIR))
    print(r.stdout)
    assert r.returncode == 0 and "adapter check ok" in r.stdout, r.stdout + r.stderr
