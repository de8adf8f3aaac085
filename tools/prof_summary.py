#!/usr/bin/env python3
"""Summarise a gpu_job.sh run: the bench JSON line and the rocprofv3 kernel statistics.
usage: python tools/prof_summary.py gpurun_out/TAG [n_kernels]"""
import csv
import json
import os
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 14
for line in open(os.path.join(d, "bench.log")):
    if line.startswith("{"):
        b = json.loads(line)
        keys = ["value", "ms_per_step", "ms_per_gn_iter", "gn_iterations", "icp_kernel_ms", "index_build_ms",
                "cov_kernel_ms"]
        print({k: round(b[k], 3) for k in keys if k in b}, "roofline frac", round(b["roofline"]["frac"], 4))
stats = os.path.join(d, "prof", "run_kernel_stats.csv")
if os.path.exists(stats):
    rows = list(csv.DictReader(open(stats)))
    for r in rows[:n]:
        print(f"{r['Name'][:58]:58s} calls={r['Calls']:>6s} avg_us={float(r['AverageNs']) / 1e3:9.1f} "
              f"tot_ms={float(r['TotalDurationNs']) / 1e6:8.2f} {float(r['Percentage']):5.1f}%")
