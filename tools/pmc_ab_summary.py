#!/usr/bin/env python3
"""Per-kernel-instantiation PMC summary of a tools/r6_pmc_ab_job.sh output directory: the mean
per dispatch of every counter, for every icp_ang_kernel form that ran."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
    per = defaultdict(float)
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if "icp_ang_kernel" not in r["Kernel_Name"]:
                continue
            k = r["Kernel_Name"]
            form = k[k.index("icp_ang_kernel"):k.index(">") + 1] if ">" in k else k
            per[(form, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (form, d, c), v in per.items():
        acc[form][c].append(v)
for form, cs in sorted(acc.items()):
    print(form)
    for c, vs in sorted(cs.items()):
        print(f"  {c:24s} {sum(vs) / len(vs):16.4g}  ({len(vs)} dispatches)")
    g = {c: sum(v) / len(v) for c, v in cs.items()}
    if g.get("SQ_INSTS_LDS"):
        print(f"  bank-conflict cycles per LDS instr {g.get('SQ_LDS_BANK_CONFLICT', 0) / g['SQ_INSTS_LDS']:.3f}")
    if g.get("SQ_WAVES"):
        print(f"  VALU instr per wave {g.get('SQ_INSTS_VALU', 0) / g['SQ_WAVES']:.0f}  LDS instr per wave "
              f"{g.get('SQ_INSTS_LDS', 0) / g['SQ_WAVES']:.0f}  SALU per wave {g.get('SQ_INSTS_SALU', 0) / g['SQ_WAVES']:.0f}")
