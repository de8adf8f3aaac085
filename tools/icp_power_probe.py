#!/usr/bin/env python3
"""Is the ICP kernel power- or clock-limited?  Runs the staged config-4 batch back to back for
SECONDS while a child process samples `amd-smi metric` (power, clocks); prints the ICP kernel time
per launch and the samples.  Reads the metrics only (no settings change).
usage: python tools/icp_power_probe.py [seconds]"""
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpg-slam_amd"))

secs = float(sys.argv[1]) if len(sys.argv) > 1 else 6.0
out = os.path.join(ROOT, "gpurun_out", "power_samples.txt")
os.makedirs(os.path.dirname(out), exist_ok=True)
# the sampler starts before this process touches the GPU (a child, never an exec)
sampler = subprocess.Popen(
    ["bash", "-c", f"end=$(( $(date +%s) + {int(secs) + 6} )); while [ $(date +%s) -lt $end ]; do date +%s.%N; "
     "timeout 5 amd-smi metric -g 0 -p -c 2>&1 | grep -v '^$'; sleep 0.1; done"],
    stdout=open(out, "w"), stderr=subprocess.STDOUT)

from dpgslam import _abi, api, synth  # noqa: E402

w = synth.generate("config4")
p = _abi.default_icp_params()
with api.Context(0) as ctx:
    ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
    ctx.icp_prepare(w.edges, w.est, p)
    ctx.icp_run(compute_cov=False)
    ctx.synchronize()
    time.sleep(1.0)   # idle samples first
    t_on = time.time()
    ms = []
    while time.time() - t_on < secs:
        ctx.icp_run(compute_cov=False)
        ctx.synchronize()
        ms.append(ctx.icp_kernel_ms())
    t_off = time.time()
    print(f"ICP back to back {len(ms)} launches: median {np.median(ms):.3f} ms, first {ms[0]:.3f}, "
          f"last {ms[-1]:.3f}, min {min(ms):.3f}; busy window {t_on:.2f} .. {t_off:.2f}")
time.sleep(1.0)
sampler.wait(timeout=60)
print(open(out).read()[-6000:])
