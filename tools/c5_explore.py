"""Config-5 workload exploration (GPU box): for several generator settings, run executeDPG after
every node of the later passes (ground-truth poses) and report per pass the mean candidate /
submap-node counts, the active-node fraction at the end of the pass and the ms per call -- to pick
a dynamic workload whose map does not collapse.  usage: python tools/c5_explore.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dpg-slam_amd")]
import numpy as np  # noqa: E402

from dpgslam import api, synth  # noqa: E402

VARIANTS = {
    "A_w40_fov360_flip": dict(world_size=40.0),
    "N0_w40_fov360_flip": dict(world_size=40.0, range_noise=0.0),
    "N2_w40_fov360_flip": dict(world_size=40.0, range_noise=0.002),
    "N5_w40_fov360_flip": dict(world_size=40.0, range_noise=0.005),
    "N2_w64_fov270_flip": dict(world_size=64.0, fov_deg=270.0, n_boxes=48, range_noise=0.002),
    "N0_w64_fov270_flip": dict(world_size=64.0, fov_deg=270.0, n_boxes=48, range_noise=0.0),
}


def main():
    names = sys.argv[1:] or list(VARIANTS)
    ctx = api.Context(0)
    for name in names:
        t = time.time()
        w = synth.make_dynamic(**VARIANTS[name])
        gen = time.time() - t
        g = api.DpgStore(ctx, w.ranges, w.geom)
        out = {"variant": name, "gen_s": round(gen, 1), "removed_boxes_per_pass":
               [int((w.present[p - 1] & ~w.present[p]).sum()) for p in range(1, len(w.present))], "passes": []}
        for p in range(1, len(w.pass_start) - 1):
            cand, sub, ms, rem = [], [], [], 0
            for v in range(int(w.pass_start[p]), int(w.pass_start[p + 1])):
                st = g.execute_dpg(v + 1, int(v - w.pass_start[p] + 1), w.est[:v + 1])
                cand.append(st.n_candidates)
                sub.append(st.n_submap_nodes)
                ms.append(st.ms_total)
                rem += st.n_removed
            _, _, na = g.fetch()
            past = int(w.pass_start[p + 1])
            cand = np.asarray(cand)
            out["passes"].append({"pass": p, "cand_mean": float(cand.mean()), "cand_p10": float(np.percentile(cand, 10)),
                                  "cand_ge50": float((cand >= 50).mean()), "submap_mean": float(np.mean(sub)),
                                  "removed_pts": int(rem), "active_frac_end": float(na[:past].mean()),
                                  "ms_mean": float(np.mean(ms)), "ms_p90": float(np.percentile(ms, 90))})
            print(json.dumps(out["passes"][-1]), file=sys.stderr, flush=True)
        g.close()
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
