#!/usr/bin/env python3
"""The bench step's GPU timeline from a rocprofv3 kernel trace (run_kernel_trace.csv): for each step
(from one ICP kernel to the next) the span, the busy time of every kernel class, and the idle gaps
of the GN phase (from the end of the ICP kernel to the end of the step's last kernel).
usage: python tools/gn_timeline.py gpurun_out/TAG/prof [steps]"""
import collections
import csv
import os
import sys

d = sys.argv[1]
nshow = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
icp = [i for i, k in enumerate(ks) if "icp_ang_kernel" in k[2]]
print(f"{len(ks)} kernels, {len(icp)} ICP launches")
for si in range(max(0, len(icp) - 1 - nshow), len(icp) - 1):
    a, b = icp[si], icp[si + 1]
    step = ks[a:b]
    # the step ends with its last kernel before the next ICP (the host's gap before the next step is not GPU time)
    t0, t_icp_end = step[0][0], step[0][1]
    t_end = max(e for _, e, _ in step)
    busy = collections.defaultdict(float)
    cnt = collections.Counter()
    for s, e, n in step:
        key = n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0].split("<")[0]
        busy[key] += (e - s) / 1e3
        cnt[key] += 1
    # GN phase: the union of kernel intervals after the ICP kernel
    iv = sorted((s, e) for s, e, n in step[1:])
    union, cur_s, cur_e, gaps = 0, None, None, []
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                union += cur_e - cur_s
                gaps.append((s - cur_e) / 1e3)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        union += cur_e - cur_s
    first_after = iv[0][0] if iv else t_icp_end
    print(f"\nstep {si}: span {(t_end - t0) / 1e3:.1f} us, ICP {(t_icp_end - t0) / 1e3:.1f} us, "
          f"gap ICP->next {(first_after - t_icp_end) / 1e3:.1f} us, after-ICP span {(t_end - first_after) / 1e3:.1f} us, "
          f"busy (union) {union / 1e3:.1f} us, idle {sum(gaps):.1f} us in {len(gaps)} gaps "
          f"(>20 us: {sum(g for g in gaps if g > 20):.1f} us in {sum(1 for g in gaps if g > 20)})")
    for k, v in sorted(busy.items(), key=lambda x: -x[1]):
        print(f"   {k[:40]:40s} n={cnt[k]:4d} busy {v:8.1f} us")
    if si == len(icp) - 2:
        print("   largest gaps (us) after:", sorted(((round((iv[j + 1][0] - max(e for _, e in iv[:j + 1])) / 1e3, 1),
                                                         [n for s, e, n in step[1:] if (s, e) == iv[j]][0].replace("void ", "").replace("(anonymous namespace)::", "")[:24])
                                                        for j in range(len(iv) - 1)), reverse=True)[:12])
