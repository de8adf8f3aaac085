#!/usr/bin/env python3
"""Summarise a tools/pmc_job.sh run: per-kernel mean of every counter over its dispatches, the HBM
traffic per launch, corrected as MI355X_MICROARCH.md "HBM" prescribes (FETCH_SIZE is in KiB and
reads 1/2 of a streamed read on gfx950 -> x2; WRITE_SIZE in KiB), and SQ fractions:
  wait_any     = SQ_WAIT_ANY / SQ_WAVE_CYCLES         (resident wave-cycles parked at waitcnt/barrier)
  active_inst  = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  clock_ghz    = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration (effective clock of the pass)
  valu_issue   = SQ_INSTS_VALU x 2 cycles / (duration x clock x 1024 SIMDs)   (wave64 VALU = 2 cycles)
  lds_issue    = SQ_INSTS_LDS x 4 cycles / (duration x clock x 256 CUs)      (ds_read_b128 = 4 cycles)
  lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS   (extra LDS cycles per LDS instruction)
Durations come from the kernel trace recorded in the same pass as the SQ counters.
usage: python tools/pmc_summary.py gpurun_out/TAG OUT.md [OUT_traffic.json]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def kname(n: str) -> str:
    return n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]


d, out_md = sys.argv[1], sys.argv[2]
out_json = sys.argv[3] if len(sys.argv) > 3 else None
acc = defaultdict(list)
dur = defaultdict(lambda: defaultdict(list))   # pass -> kernel -> durations (ns)
for f in sorted(glob.glob(os.path.join(d, "*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        acc[(kname(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
for f in sorted(glob.glob(os.path.join(d, "*", "run_kernel_trace.csv"))):
    ps = os.path.basename(os.path.dirname(f))
    for r in csv.DictReader(open(f)):
        dur[ps][kname(r["Kernel_Name"])].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
kernels = sorted({k for k, _ in acc})
lines = [f"# PMC summary of `{d}` (mean per dispatch)", "", "| kernel | counter | dispatches | mean |", "|---|---|---|---|"]
for k in kernels:
    for (kk, c), v in sorted(acc.items()):
        if kk == k:
            lines.append(f"| `{k}` | {c} | {len(v)} | {sum(v) / len(v):.6g} |")
traffic, fracs = {}, {}
mean = lambda k, c: (sum(acc[(k, c)]) / len(acc[(k, c)])) if acc.get((k, c)) else None   # noqa: E731
for k in kernels:
    fe, wr = mean(k, "FETCH_SIZE"), mean(k, "WRITE_SIZE")
    if fe is not None and wr is not None:
        traffic[k] = (2.0 * fe + wr) * 1024.0
    wc = mean(k, "SQ_WAVE_CYCLES")
    if wc:
        fr = {}
        if mean(k, "SQ_WAIT_ANY") is not None:
            fr["wait_any"] = mean(k, "SQ_WAIT_ANY") / wc
        if mean(k, "SQ_ACTIVE_INST_ANY") is not None:
            fr["active_inst"] = mean(k, "SQ_ACTIVE_INST_ANY") / wc
        ds = dur.get("sq", {}).get(k)
        gui = mean(k, "GRBM_GUI_ACTIVE")
        if ds and gui:
            t_ns = sum(ds) / len(ds)
            clk = gui / 8.0 / t_ns   # GHz
            fr["duration_ms"] = t_ns * 1e-6
            fr["clock_ghz"] = clk
            if mean(k, "SQ_INSTS_VALU") is not None:
                fr["valu_issue"] = mean(k, "SQ_INSTS_VALU") * 2.0 / (t_ns * clk * 1024.0)
            if mean(k, "SQ_INSTS_LDS") is not None:
                fr["lds_issue"] = mean(k, "SQ_INSTS_LDS") * 4.0 / (t_ns * clk * 256.0)
        if mean(k, "SQ_LDS_BANK_CONFLICT") is not None and mean(k, "SQ_INSTS_LDS"):
            fr["lds_conflict"] = mean(k, "SQ_LDS_BANK_CONFLICT") / mean(k, "SQ_INSTS_LDS")
        fracs[k] = fr
lines += ["", "HBM traffic per launch = (2 x FETCH_SIZE + WRITE_SIZE) KiB x 1024:", ""]
lines += [f"* `{k}`: {t / 1e6:.1f} MB" for k, t in traffic.items()]
lines += ["", "SQ fractions (see tools/pmc_summary.py for the definitions):", ""]
lines += [f"* `{k}`: " + ", ".join(f"{a} {b:.3g}" for a, b in fr.items()) for k, fr in fracs.items() if fr]
open(out_md, "w").write("\n".join(lines) + "\n")
if out_json:
    counts = {k: {c: mean(k, c) for (kk, c) in acc if kk == k} for k in kernels}
    meta = {}
    for name in ("src.sha256", "git.sha"):   # written by tools/pmc_job.sh beside the passes
        f = os.path.join(d, name)
        if os.path.exists(f):
            meta["src_sha256" if name == "src.sha256" else "git_sha"] = open(f).read().split()[0]
    json.dump({"source": os.path.basename(os.path.normpath(d)), **meta, "traffic_bytes_per_launch": traffic,
               "sq_fractions": fracs, "counts": counts}, open(out_json, "w"), indent=1)
print("\n".join(l for l in lines if l.startswith("* `icp") or l.startswith("* `chol")))
