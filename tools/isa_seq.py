"""Memory-op / wait sequence of selected kernels in the built library (offline ISA audit).

usage: python tools/isa_seq.py <mangled-name regex> [--full]
Prints, per matching kernel, the vector-memory loads / stores / LDS-DMA, s_waitcnt, s_barrier and
branch lines in program order (runs of identical lines collapsed), so a wait that drains the
memory pipe between an epilogue's loads and stores is visible without reading the whole listing."""
import re
import subprocess
import sys
import os

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from skeletondiffusion_amd import isa_check  # noqa: E402

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "skeletondiffusion_amd", "libskeldiff.so")
KEEP = re.compile(r"\b(global_load\w*|global_store\w*|buffer_\w+|s_waitcnt\b.*|s_barrier|s_cbranch\w*|s_branch|global_atomic\w*|s_endpgm)")


def listing():
    out = []
    for i, (_t, b) in enumerate(isa_check.code_objects(LIB)):
        path = f"/tmp/isa/co{i}.o"
        with open(path, "wb") as f:
            f.write(b)
        out.append(subprocess.run([isa_check._tool("llvm-objdump"), "-d", "--mcpu=gfx950", path], check=True,
                                  capture_output=True, text=True).stdout)
    return "\n".join(out)


def main():
    pat = re.compile(sys.argv[1])
    full = "--full" in sys.argv
    for f in re.split(r"\n(?=[0-9a-f]{16} <)", listing()):
        m = re.match(r"[0-9a-f]+ <(\S+)>:", f)
        if not m or not pat.search(m.group(1)):
            continue
        name = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
        print("==", name[:160], f"({len(f.splitlines())} lines)")
        prev, n = None, 0
        for line in f.splitlines():
            ins = line.split("//")[0].strip()
            k = KEEP.search(ins)
            if not k:
                continue
            key = ins if full else re.sub(r"\s+v\[?[\d:]+\]?.*$", "", ins) if not ins.startswith("s_") else ins
            if key == prev:
                n += 1
                continue
            if prev is not None:
                print(f"  {prev}" + (f"  x{n}" if n > 1 else ""))
            prev, n = key, 1
        if prev is not None:
            print(f"  {prev}" + (f"  x{n}" if n > 1 else ""))


if __name__ == "__main__":
    main()
