#!/usr/bin/env python3
"""Concurrency view of a rocprofv3 kernel trace of bench.py with row chains: over the span of the
timed sampler launches, the union of kernel intervals (GPU busy), the sum of kernel durations
(overlap = sum / union) and a CU-occupancy estimate (each launch holds min(WGs, 256) CUs for its
duration; one workgroup per CU for k_gl4).  Usage: python tools/trace_overlap.py <run_kernel_trace.csv>"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ev = []
for r in rows:
    n = r["Kernel_Name"]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    grid = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
    wg = int(r.get("Workgroup_Size") or r.get("Workgroup_Size_X") or 256)
    ev.append((s, e, n.split("(")[0].replace("void ", ""), max(1, grid // max(wg, 1))))
ev.sort()
# timed region: the densest window = from the first to the last chained-tile launch (k_gl4<16, 8, 1, 2)
ch = [x for x in ev if "k_gl4<16, 8, 1, 2" in x[2]]
if not ch:
    ch = ev
t0, t1 = ch[0][0], max(x[1] for x in ch)
sel = [x for x in ev if x[0] >= t0 and x[1] <= t1]
# union
busy, cur_s, cur_e = 0, None, None
for s, e, _, _ in sel:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = t1 - t0
tot = sum(e - s for s, e, _, _ in sel)
occ = sum((e - s) * min(w, 256) / 256 for s, e, _, w in sel)
print(f"span {span/1e6:.2f} ms, launches {len(sel)}, busy(union) {busy/span*100:.1f} %, "
      f"sum(dur)/span {tot/span:.2f}, CU-occupancy estimate {occ/span*100:.1f} %")
agg = defaultdict(lambda: [0, 0.0, 0.0, 0])
for s, e, n, w in sel:
    a = agg[n]
    a[0] += 1
    a[1] += e - s
    a[2] += (e - s) * min(w, 256) / 256
    a[3] = w
for n, (c, d, o, w) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{n[:70]:70s} n={c:6d} avg={d/c/1e3:8.1f} us  WGs={w:5d}  share(dur) {d/tot*100:5.1f} %  CU-time {o/span*100:5.1f} %")
