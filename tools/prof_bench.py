#!/usr/bin/env python3
"""Summarise a tools/prof_bench.sh run into profiles/<tag>/summary.md, copy the rocprofv3 kernel
stats there, and record the per-layer HBM traffic in profiles/pmc_traffic.json under
"<config>|<route bits>" (the kernels the bench's call launched, bench.py config.route_bits).

Per kernel (PMC passes, averaged over its dispatches): HBM read = 2 x FETCH_SIZE (gfx950 counts
half the bytes of a wide coalesced stream, MI355X_MICROARCH.md §HBM), write = WRITE_SIZE (exact
for 16-B-per-lane stores), MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1,024
SIMDs): the share of the dispatch's SIMD-cycles the matrix pipes were busy.
One graph-linear layer = one GEMM-phase dispatch (k_gl4t / k_gl4y) + one mixing-phase dispatch
(k_gl4 MODE 2 / 3) on the split routes, or one k_gl4 dispatch on the one-kernel route.
usage: python tools/prof_bench.py gpurun_out/prof_<tag> <tag> [config]"""
import csv
import json
import os
import re
import shutil
import sys
from collections import defaultdict

src, tag = sys.argv[1], sys.argv[2]
config = sys.argv[3] if len(sys.argv) > 3 else "amass16"
HERE = os.path.dirname(os.path.abspath(__file__))
dst = os.path.join(os.path.dirname(HERE), "profiles", tag)
os.makedirs(dst, exist_ok=True)


def short(name):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", n)


def kind(name):
    n = short(name)
    if "k_gl4t" in n:
        return "gemm_tiled"
    if "k_gl4y" in n:
        return "gemm_wave"
    m = re.match(r"sd::k_gl4<(.*)>", n)
    if m:
        args = m.group(1).split(",")
        # <J, NW, RT, CT, RMS, MODE, PREC, STG> (ABI 3+); rounds 1-5 had two more arguments, MODE 7th
        mode = int(args[5]) if len(args) == 8 else int(args[6]) if len(args) > 6 else 0
        return {0: "one_kernel", 1: "fused_attention", 2: "mix_phase", 3: "attn_phase", 4: "one_kernel"}.get(mode, "other")
    if "k_gl5_mix" in n:  # J > 21: the mixing pass of a plain layer
        return "mix_phase"
    if "k_attention" in n:  # the attention kernel (k_attention_mix: with to_qkv's mixing)
        return "attn_phase"
    if "k_update" in n:
        return "update"
    return "other"


def bench_line(path):
    for line in open(path):
        if line.startswith("{"):
            return json.loads(line)
    return None


stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "run_kernel_stats.csv"))
b = bench_line(os.path.join(src, "trace.log"))
lines = [f"# rocprofv3 profile `{tag}`: `bench.py` ({config})", ""]
if b:
    lines += [f"Bench line of the profiled command: {b['value']:.0f} futures/s (profiled run), route "
              f"`{b['config']['route']}`, row chains {b['config']['row_chains']}, kernels {b['config']['kernels']}.", ""]
lines += ["## Kernel stats (`rocprofv3 --kernel-trace --stats`, `run_kernel_stats.csv`)", "",
          "| kernel | calls | avg µs | share % |", "|---|---|---|---|"]
for s in stats[:14]:
    lines.append(f"| `{short(s['Name'])[:90]}` | {s['Calls']} | {float(s['AverageNs']) / 1e3:.1f} | "
                 f"{float(s['Percentage']):.2f} |")

pmc = defaultdict(lambda: defaultdict(list))  # kernel short name -> counter -> values
for i in (1, 2, 3):
    path = os.path.join(src, f"pmc{i}", "run_counter_collection.csv")
    if not os.path.exists(path):
        continue
    for r in csv.DictReader(open(path)):
        pmc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
pm = bench_line(os.path.join(src, "pmc1.log"))
rows = pm["config"]["rows_per_gpu"] if pm else None
route_bits = pm["config"].get("route_bits") if pm else None
if pmc:
    lines += ["", "## PMC per dispatch (separate passes; T = 4 run of the same configuration)", "",
              "| kernel | dispatches | HBM read MB (2 x FETCH) | write MB | MFMA busy % of SIMD-cycles | wait-inst % | wait % |",
              "|---|---|---|---|---|---|---|"]
    layer_bytes, layers = 0.0, 0
    for k, c in sorted(pmc.items(), key=lambda kv: -sum(kv[1].get("FETCH_SIZE", [0]))):
        avg = {n: sum(v) / len(v) for n, v in c.items()}
        nd = max(len(v) for v in c.values())
        rd = 2 * avg.get("FETCH_SIZE", 0) * 1024 / 1e6
        wr = avg.get("WRITE_SIZE", 0) * 1024 / 1e6
        gui = avg.get("GRBM_GUI_ACTIVE", 0) / 8  # summed over the 8 XCDs
        mfma = avg.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (gui * 1024) * 100 if gui else float("nan")
        wave = avg.get("SQ_WAVE_CYCLES", 0)
        wi = avg.get("SQ_WAIT_INST_ANY", 0) / wave * 100 if wave else float("nan")
        wa = avg.get("SQ_WAIT_ANY", 0) / wave * 100 if wave else float("nan")
        lines.append(f"| `{k[:80]}` | {nd} | {rd:.1f} | {wr:.1f} | {mfma:.1f} | {wi:.1f} | {wa:.1f} |")
        kd = kind(k)
        if kd in ("gemm_tiled", "gemm_wave", "one_kernel", "fused_attention", "mix_phase", "attn_phase"):
            tot = sum(c.get("FETCH_SIZE", [])) * 2 * 1024 + sum(c.get("WRITE_SIZE", [])) * 1024
            layer_bytes += tot
            if kd in ("gemm_tiled", "gemm_wave", "one_kernel", "fused_attention"):
                layers += len(c.get("FETCH_SIZE", []))
    if layers:
        per = layer_bytes / layers
        lines += ["", f"HBM traffic per graph-linear layer launch: **{per / 1e6:.1f} MB** "
                      f"({layers} layer launches in the FETCH / WRITE passes)."]
        if b:
            alg = b["roofline"]["algorithmic_bytes_per_launch"]
            lines.append(f"Algorithmic bytes per layer launch: {alg / 1e6:.1f} MB -> traffic / algorithmic = "
                         f"{per / alg:.2f}.")
        tf = os.path.join(os.path.dirname(HERE), "profiles", "pmc_traffic.json")
        db = json.load(open(tf)) if os.path.exists(tf) else {}
        db = {k: v for k, v in db.items() if "|" in k}  # keys of the old format (config only) are stale
        db[f"{config}|{route_bits}"] = {"rows": rows, "hbm_bytes_per_layer_launch": per,
                                        "source": f"profiles/{tag}/summary.md (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, "
                                                  f"2 x FETCH + WRITE per layer launch)"}
        json.dump(db, open(tf, "w"), indent=1)
open(os.path.join(dst, "summary.md"), "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
