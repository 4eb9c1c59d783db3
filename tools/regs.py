"""Per-kernel register / spill / occupancy table for one HIP source (hipcc resource remarks).
Usage: python tools/regs.py skeletondiffusion_amd/csrc/sd_graph_linear_v4.hip [filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", "-Rpass-analysis=kernel-resource-usage",
                      src, "-o", "/tmp/_regs.o"], capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": subprocess.run(["c++filt"], input=t.split(":", 1)[1].strip(), capture_output=True,
                                      text=True).stdout.strip() if True else t}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    if flt in r["name"]:
        print(f"{r['name'][:60]:60s} V={r.get('VGPRs')} A={r.get('AGPRs')} spillV={r.get('VGPRs Spill')} "
              f"occ={r.get('Occupancy [waves/SIMD]')} scratch={r.get('ScratchSize [bytes/lane]')}")
