"""Shared pytest setup: markers, import paths, the oracle build, and cached workloads."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "dpg-slam_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); parity tests through the C ABI")
    config.addinivalue_line("markers", "slow: full-size (config 4) case")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


_WL = {}


@pytest.fixture(scope="session")
def workload():
    from dpgslam import synth

    def get(name):
        if name not in _WL:
            _WL[name] = synth.generate(name)
        return _WL[name]
    return get


@pytest.fixture(scope="session")
def ctx():
    """A GPU context; on a GPU box a missing/broken library must FAIL, not skip."""
    from dpgslam import api
    try:   # torch's HIP runtime first (as bench.py does): tests hand torch device buffers to libdpg
        import torch
        if torch.cuda.device_count() > 0:
            torch.cuda.init()
    except ImportError:
        pass
    c = api.Context(0)
    yield c
    c.close()


def angle_wrap(a):
    return np.arctan2(np.sin(a), np.cos(a))
