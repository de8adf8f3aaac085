"""Debug driver: tests/test_slam.py's lockstep run with progress prints and forced collections."""
import gc
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpg-slam_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402


def main():
    from dpgslam import api, synth
    from dpgslam.slam import DpgSLAM
    from slam_lockstep import LockstepBackend
    print("import ok", flush=True)
    w = synth.make_dynamic(n_passes=2, nodes_per_pass=14, n_beams=360, world_size=16.0, range_max=8.0, n_boxes=6, seed=9)
    ctx = api.Context(0)
    print("ctx ok", flush=True)
    be = LockstepBackend(ctx, every=1, dpg_every=1, sweep_sample=10 ** 6)
    print("backend ok", flush=True)
    gc.collect()
    sg = DpgSLAM(backend=be)
    be.clouds_of = lambda: sg.clouds
    rng = np.random.default_rng(3)
    P = len(w.pass_start) - 1
    for p in range(P):
        if p:
            print("increment pass", flush=True)
            sg.incrementPassNumber()
            gc.collect()
        for v in range(int(w.pass_start[p]), int(w.pass_start[p + 1])):
            odom = w.est[v].astype(np.float64) + rng.normal(0, [0.01, 0.01, 0.002])
            sg.ObserveOdometry(odom[:2].astype(np.float32), np.float32(odom[2]))
            sg.ObserveLaser(w.ranges[v], 0.0, float(w.geom[v, 2]), float(w.geom[v, 0]), float(w.geom[v, 1]))
            print(f"reading {v}: nodes {len(sg.poses)} checked {be.checked}", flush=True)
            gc.collect()
    print("done", be.checked, be.max_pose_diff, flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
