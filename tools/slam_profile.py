#!/usr/bin/env python3
"""cProfile of the DpgSLAM driver's per-node path on the GPU backend (config 5's patrol workload,
2 passes x 600 readings): where the host time outside the C calls goes.
usage: python tools/slam_profile.py [steps]"""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpg-slam_amd")]
from dpgslam import synth  # noqa: E402
from dpgslam.slam import DpgSLAM  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 600
w = synth.make_patrol(n_passes=2, steps=steps)
slam = DpgSLAM(backend="gpu")
amin, amax, rmax = (float(x) for x in w.geom[0])


def drive(p0, p1):
    for p in range(p0, p1):
        if p:
            slam.incrementPassNumber()
        for k in range(w.steps):
            o = w.odom[p, k]
            slam.ObserveOdometry(o[:2], o[2])
            slam.ObserveLaser(w.ranges[p * w.steps + k], 0.0, rmax, amin, amax)


drive(0, 1)   # warm-up pass (not profiled)
pr = cProfile.Profile()
pr.enable()
drive(1, 2)
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
st.sort_stats("cumtime").print_stats(25)
