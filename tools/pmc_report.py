"""Summarise tools/pmc_gl.sh / tools/pmc_kernel.sh output: MFMA utilisation, stall split,
instruction mix, LDS bank conflicts.
usage: python tools/pmc_report.py [--kernel REGEX] [--dir PATTERN] tag [tag ...]
(defaults: the graph-linear kernels, gpurun_out/pmc_gl_<tag>)"""
import argparse
import collections
import csv
import glob
import re

ap = argparse.ArgumentParser()
ap.add_argument("--kernel", default=r"k_gl|k_graph_linear")
ap.add_argument("--dir", default="gpurun_out/pmc_gl_{tag}")
ap.add_argument("--raw", action="store_true", help="also print every counter's per-dispatch average")
ap.add_argument("tags", nargs="+")
args = ap.parse_args()
kpat = re.compile(args.kernel)

for tag in args.tags:
    vals = collections.defaultdict(list)
    for f in sorted(glob.glob(args.dir.format(tag=tag) + "/p*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if not kpat.search(r["Kernel_Name"]):
                continue
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    a = {k: sum(v) / len(v) for k, v in vals.items()}
    w = a.get("SQ_WAVE_CYCLES", float("nan"))  # percentages of wave cycles: nan without that counter
    gui = a.get("GRBM_GUI_ACTIVE", 8) / 8          # summed over the 8 XCDs
    print(f"===== {tag}: kernel {gui / 2.4e3:.1f} us (at 2.4 GHz)  MFMA util "
          f"{a.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (gui * 1024) * 100:.1f}%  waves/SIMD {w * 4 / (gui * 1024):.2f}")
    print(f"  wait_any {a.get('SQ_WAIT_ANY', 0) / w * 100:.1f}%  wait_inst {a.get('SQ_WAIT_INST_ANY', 0) / w * 100:.1f}%"
          f"  active {a.get('SQ_ACTIVE_INST_ANY', 0) / w * 100:.1f}%")
    hit = a.get("TCC_HIT_sum", 0) / max(a.get("TCC_HIT_sum", 0) + a.get("TCC_MISS_sum", 0), 1)
    print(f"  insts VALU {a.get('SQ_INSTS_VALU', 0):,.0f} LDS {a.get('SQ_INSTS_LDS', 0):,.0f} VMEM "
          f"{a.get('SQ_INSTS_VMEM', 0):,.0f} SALU {a.get('SQ_INSTS_SALU', 0):,.0f}  LDS bank conflicts "
          f"{a.get('SQ_LDS_BANK_CONFLICT', 0):,.0f}  L2 hit {hit * 100:.1f}%")
    if "SQ_LDS_IDX_ACTIVE" in a or "SQ_INSTS_MFMA" in a:
        print(f"  LDS array cycles {a.get('SQ_LDS_IDX_ACTIVE', 0):,.0f} (bank-conflict share "
              f"{a.get('SQ_LDS_BANK_CONFLICT', 0) / max(a.get('SQ_LDS_IDX_ACTIVE', 0), 1) * 100:.1f}%)  LDS-issue stall "
              f"{a.get('SQ_WAIT_INST_LDS', 0) / w * 100:.1f}% of wave cycles  MFMA insts {a.get('SQ_INSTS_MFMA', 0):,.0f}")
    if args.raw:
        for k in sorted(a):
            print(f"    {k:32s} {a[k]:16,.0f}  ({a[k] / w * 100:6.1f}% of wave cycles)" if k.startswith("SQ_")
                  else f"    {k:32s} {a[k]:16,.0f}")
    if "FETCH_SIZE" in a:
        print(f"  HBM/MALL bytes per launch: fetch {2 * a['FETCH_SIZE'] * 1024 / 1e6:.1f} MB (2x FETCH_SIZE, gfx950)"
              f"  write {a.get('WRITE_SIZE', 0) * 1024 / 1e6:.1f} MB")
