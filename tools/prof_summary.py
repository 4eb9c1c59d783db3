#!/usr/bin/env python3
"""Summarise a tools/profile.sh run (rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes)
into profiles/<tag>_summary.md and the traffic json bench.py reads.

HBM bytes per launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024: on gfx950 FETCH_SIZE reports
half the bytes of a wide coalesced stream (MI355X_MICROARCH.md §HBM), so it is doubled;
WRITE_SIZE is exact for 16-B-per-lane stores and uncalibrated for other widths (noted).
Usage: python tools/prof_summary.py gpurun_out/prof_r01_v2 r01_v2 [rows J]
"""
import csv
import json
import os
import sys
from collections import defaultdict

src, tag = sys.argv[1], sys.argv[2]
rows_b = int(sys.argv[3]) if len(sys.argv) > 3 else 3200
J = int(sys.argv[4]) if len(sys.argv) > 4 else 16
H, D, HID = 192, 96, 256


def short(name):
    return name.split("(")[0].replace("void ", "")


stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
trace = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))))

# graph-linear layer shape from the grid: ntile_c * ntile_r workgroups of 256 threads
ntile_r = (rows_b + 63) // 64
by_shape = defaultdict(list)
for r in trace:
    n = r["Kernel_Name"]
    if "k_gl2" not in n and "k_graph_linear" not in n and "k_gl3" not in n and "k_gl4" not in n:
        continue
    wgs = int(r.get("Grid_Size") or r["Grid_Size_X"]) // 256
    if "k_gl4t" in n or "k_gl4y" in n:  # split-route phase 1: N from its template / not recoverable
        targs = [t.strip() for t in n.split("<")[1].split(">")[0].split(",")]
        if "k_gl4y" in n:
            nt, NT = 0, 0
        else:  # <RMS, PREC, CT, NCH, ROWMAJOR, PF>: 4 row tiles x CT column tiles of one node
            nt, NT = wgs // ((((rows_b + 31) // 32 + 3) // 4) * J), 32 * int(targs[2])
    elif "k_gl4" in n:  # <J, NW, RT, CT, RMS, DBG, MODE>: tile 32 RT rows x 32 CT columns, NW * 64 threads
        targs = [t.strip() for t in n.split("<")[1].split(">")[0].split(",")]
        nw, rt, ctl = int(targs[1]), int(targs[2]), int(targs[3])
        wgs = int(r.get("Grid_Size") or r["Grid_Size_X"]) // (nw * 64)
        mode = int(targs[6]) if len(targs) > 6 else 0
        nt = wgs // ((rows_b + 32 * rt - 1) // (32 * rt))
        NT = 96 if mode == 1 else 32 * ctl  # mode 1: one head (q|k|v) per column tile
    elif "k_gl3" in n:
        nt, NT = wgs // ((rows_b + 31) // 32), 32
    else:
        nt = wgs // ntile_r
        NT = 32 if ", 2, " in n.split("<")[1] else 16
    by_shape[(short(n), nt * NT)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))

# per layer (K1+K2, N) of the release Denoiser at this J
K_OF_N = {H: None, 3 * HID: H, D: H}
lines = [f"# rocprofv3 summary `{tag}` (bench.py default workload, B={rows_b} rows, J={J})", "",
         "## Kernel stats (`rocprofv3 --kernel-trace --stats`)", "",
         "| kernel | calls | avg µs | min µs | max µs | share % |", "|---|---|---|---|---|---|"]
for s in stats[:12]:
    lines.append(f"| `{short(s['Name'])[:60]}` | {s['Calls']} | {float(s['AverageNs'])/1e3:.1f} | "
                 f"{float(s['MinNs'])/1e3:.1f} | {float(s['MaxNs'])/1e3:.1f} | {float(s['Percentage']):.2f} |")
lines += ["", "## graph-linear launches by output width N (from grid size)", "",
          "| kernel | N | launches | avg µs |", "|---|---|---|---|"]
for (k, N), ds in sorted(by_shape.items()):
    lines.append(f"| `{k}` | {N} | {len(ds)} | {sum(ds)/len(ds)/1e3:.1f} |")

traffic = {}
for kind in ("fetch", "write"):
    path = os.path.join(src, f"pmc_{kind}", "run_counter_collection.csv")
    if not os.path.exists(path):
        continue
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    traffic[kind] = {k: sum(v) / len(v) for k, v in acc.items()}
if traffic:
    lines += ["", "## HBM traffic per launch (PMC, separate passes)", "",
              "| kernel | FETCH_SIZE KiB | WRITE_SIZE KiB | HBM MB (2*FETCH + WRITE) |", "|---|---|---|---|"]
    for k in sorted(traffic.get("fetch", {}), key=lambda k: -traffic["fetch"][k])[:8]:
        f = traffic["fetch"].get(k, 0.0)
        w = traffic.get("write", {}).get(k, 0.0)
        lines.append(f"| `{k[:60]}` | {f:.0f} | {w:.0f} | {(2 * f + w) * 1024 / 1e6:.1f} |")
    # the launches bench.py's roofline times (sd_profile_step: one denoise step at the full batch,
    # one stream): graph-linear dispatches whose grid covers all rows_b rows.  With row chains the
    # timed sampler's launches cover a third of the rows each and are summarised separately.
    full = defaultdict(lambda: [0.0, 0.0, 0])  # kernel -> [fetch sum, write sum, n]
    for kind, col in (("fetch", 0), ("write", 1)):
        path = os.path.join(src, f"pmc_{kind}", "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        for r in csv.DictReader(open(path)):
            n = r["Kernel_Name"]
            if "k_gl4" not in n or "k_gl4y" in n:
                continue
            targs = [t.strip() for t in n.split("<")[1].split(">")[0].split(",")]
            if "k_gl4t" in n:  # tiled split route: one k_gl4t dispatch per graph-linear layer
                full["split route (k_gl4t + k_gl4 MODE 2 / 3)"][col] += float(r["Counter_Value"])
                if col == 0:
                    full["split route (k_gl4t + k_gl4 MODE 2 / 3)"][2] += 1
                continue
            nw, rt, mode = int(targs[1]), int(targs[2]), int(targs[6])
            if mode >= 2:  # the split route's phase 2: bytes of the layer its k_gl4t dispatch counted
                full["split route (k_gl4t + k_gl4 MODE 2 / 3)"][col] += float(r["Counter_Value"])
                continue
            wgs = int(r["Grid_Size"]) // (nw * 64)
            ntile_r = (rows_b + 32 * rt - 1) // (32 * rt)
            if wgs < ntile_r or wgs % ntile_r:
                continue  # a row-chain launch
            full[short(n)][col] += float(r["Counter_Value"])
            if col == 0:
                full[short(n)][2] += 1
    gl = [k for k in traffic.get("fetch", {}) if "k_gl" in k or "k_graph_linear" in k]
    if full:
        tot_n = sum(v[2] for v in full.values())
        avg = sum((2 * v[0] + v[1]) * 1024 for v in full.values()) / max(tot_n, 1)
        lines += ["", "## full-batch graph-linear launches (the launches bench.py's roofline times)", "",
                  "| kernel | launches | HBM MB per launch (2*FETCH + WRITE) |", "|---|---|---|"]
        for k, v in full.items():
            lines.append(f"| `{k[:60]}` | {v[2]} | {(2 * v[0] + v[1]) * 1024 / max(v[2], 1) / 1e6:.1f} |")
        out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "pmc_traffic.json")
        data = json.load(open(out)) if os.path.exists(out) else {}
        data["amass16"] = {"graph_linear_bytes_per_launch": avg, "source": tag,
                           "note": "2*FETCH_SIZE + WRITE_SIZE per launch, averaged over the full-batch "
                                   "graph-linear launches of sd_profile_step (the launches the roofline times)"}
        json.dump(data, open(out, "w"), indent=1)
        lines += ["", f"full-batch graph-linear average HBM bytes per launch: {avg/1e6:.1f} MB "
                      "(written to profiles/pmc_traffic.json)"]
    elif gl:
        calls = {short(s["Name"]): int(s["Calls"]) for s in stats}
        tot_calls = sum(calls.get(k, 0) for k in gl)
        avg = sum((2 * traffic["fetch"][k] + traffic.get("write", {}).get(k, 0.0)) * 1024 * calls.get(k, 0)
                  for k in gl) / max(tot_calls, 1)
        out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "pmc_traffic.json")
        data = json.load(open(out)) if os.path.exists(out) else {}
        data["amass16"] = {"graph_linear_bytes_per_launch": avg, "source": tag,
                           "note": "2*FETCH_SIZE + WRITE_SIZE, averaged over all graph-linear launches"}
        json.dump(data, open(out, "w"), indent=1)
        lines += ["", f"graph-linear average HBM bytes per launch: {avg/1e6:.1f} MB (written to profiles/pmc_traffic.json)"]
dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", f"{tag}_summary.md")
open(dst, "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
