"""Per-step timeline of a rocprofv3 kernel trace (small batches, DESIGN.md §4d'): for the last
`--steps` denoise steps of the trace, kernel busy time vs wall time, the idle gap before each
kernel, and per-kernel-name averages.  A step is delimited by the update kernel (k_update*).
usage: python tools/trace_gaps.py <kernel_trace.csv> [--steps 20]"""
import argparse
import collections
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--steps", type=int, default=20)
args = ap.parse_args()

rows = list(csv.DictReader(open(args.trace)))
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
ends = [i for i, k in enumerate(ks) if "k_update" in k[2]]
if len(ends) < args.steps + 1:
    raise SystemExit(f"only {len(ends)} update kernels in the trace")
lo, hi = ends[-args.steps - 1] + 1, ends[-1] + 1
sel = ks[lo:hi]
wall = sel[-1][1] - sel[0][0]
busy = sum(e - s for s, e, _ in sel)
gaps = [sel[i][0] - sel[i - 1][1] for i in range(1, len(sel))]
print(f"steps {args.steps}: {len(sel) / args.steps:.1f} kernels/step, wall {wall / args.steps / 1e3:.1f} us/step, "
      f"busy {busy / args.steps / 1e3:.1f} us/step, mean gap {sum(gaps) / len(gaps) / 1e3:.2f} us, "
      f"median gap {sorted(gaps)[len(gaps) // 2] / 1e3:.2f} us")
per = collections.defaultdict(list)
gap_before = collections.defaultdict(list)
for i, (s, e, n) in enumerate(sel):
    short = n.split("(")[0][-70:]
    per[short].append(e - s)
    if i:
        gap_before[short].append(s - sel[i - 1][1])
print(f"{'kernel':72s} {'/step':>6s} {'avg us':>7s} {'gap us':>7s} {'us/step':>8s}")
for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
    g = gap_before.get(k, [0])
    print(f"{k:72s} {len(v) / args.steps:6.1f} {sum(v) / len(v) / 1e3:7.2f} {sum(g) / len(g) / 1e3:7.2f} "
          f"{sum(v) / args.steps / 1e3:8.1f}")
