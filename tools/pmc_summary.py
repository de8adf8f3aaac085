#!/usr/bin/env python3
"""Summarise a tools/pmc_job.sh run: per-kernel mean of every counter over its dispatches, and the
HBM traffic of the ICP kernel per launch, corrected as MI355X_MICROARCH.md "HBM" prescribes
(FETCH_SIZE is in KiB and reads 1/2 of a streamed read on gfx950 -> x2; WRITE_SIZE in KiB).
usage: python tools/pmc_summary.py gpurun_out/TAG OUT.md [OUT_traffic.json]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

d, out_md = sys.argv[1], sys.argv[2]
out_json = sys.argv[3] if len(sys.argv) > 3 else None
acc = defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        acc[(name, r["Counter_Name"])].append(float(r["Counter_Value"]))
kernels = sorted({k for k, _ in acc})
lines = [f"# PMC summary of `{d}` (mean per dispatch)", "", "| kernel | counter | dispatches | mean |", "|---|---|---|---|"]
for k in kernels:
    for (kk, c), v in sorted(acc.items()):
        if kk == k:
            lines.append(f"| `{k}` | {c} | {len(v)} | {sum(v) / len(v):.6g} |")
traffic = {}
for k in kernels:
    fe, wr = acc.get((k, "FETCH_SIZE")), acc.get((k, "WRITE_SIZE"))
    if fe and wr:
        t = (2.0 * sum(fe) / len(fe) + sum(wr) / len(wr)) * 1024.0
        traffic[k] = t
lines += ["", "HBM traffic per launch = (2 x FETCH_SIZE + WRITE_SIZE) KiB x 1024:", ""]
lines += [f"* `{k}`: {t / 1e6:.1f} MB" for k, t in traffic.items()]
open(out_md, "w").write("\n".join(lines) + "\n")
if out_json:
    json.dump({"source": os.path.basename(os.path.normpath(d)), "traffic_bytes_per_launch": traffic}, open(out_json, "w"), indent=1)
print("\n".join(lines[-len(traffic) - 1:]))
