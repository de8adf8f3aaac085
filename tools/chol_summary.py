#!/usr/bin/env python3
"""Summarise a chol_job.sh run: harness lines, kernel stats, per-launch timing extremes.
usage: python tools/chol_summary.py gpurun_out/TAG"""
import csv
import os
import re
import sys

d = sys.argv[1]
print(open(os.path.join(d, "chol.log")).read().strip())
st = os.path.join(d, "prof", "run_kernel_stats.csv")
if os.path.exists(st):
    for r in list(csv.DictReader(open(st)))[:8]:
        print(f"{r['Name'][:50]:50s} calls={r['Calls']:>6s} avg_us={float(r['AverageNs']) / 1e3:8.1f} "
              f"tot_ms={float(r['TotalDurationNs']) / 1e6:8.2f}")
tl = os.path.join(d, "chol_timing.log")
if os.path.exists(tl):
    lines = [l for l in open(tl) if l.startswith("L")]
    spans = sorted(((float(re.search(r"span\s+([\d.]+)", l).group(1)), l.strip()) for l in lines), reverse=True)
    for sp, l in spans[:8]:
        print(l[:170])
    print([l for l in open(tl) if l.startswith("sum")][0].strip(), f"({len(lines)} launches)")
