"""Offline audit: per kernel of the built library, the s_waitcnt vmcnt(N) instructions that can only
be waiting for STORES (since the previous vmcnt wait, only stores were issued and N is below their
count) -- the compiler's wait before it overwrites a pending store's data or address registers.
usage: python tools/isa_store_waits.py [name regex]"""
import re
import subprocess
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_seq  # noqa: E402


def main():
    pat = re.compile(sys.argv[1] if len(sys.argv) > 1 else ".")
    rows = []
    for f in re.split(r"\n(?=[0-9a-f]{16} <)", isa_seq.listing()):
        m = re.match(r"[0-9a-f]+ <(\S+)>:", f)
        if not m or not pat.search(m.group(1)):
            continue
        loads = stores = 0
        bad = 0
        for line in f.splitlines():
            ins = line.split("//")[0].strip()
            if re.match(r"(global_load|buffer_load|scratch_load|global_atomic\w*_rtn)", ins):
                loads += 1
            elif re.match(r"(global_store|buffer_store|scratch_store|global_atomic)", ins):
                stores += 1
            else:
                w = re.match(r"s_waitcnt.*vmcnt\((\d+)\)", ins)
                if w:
                    if loads == 0 and stores > int(w.group(1)):
                        bad += 1
                    loads = stores = 0
        if bad:
            rows.append((bad, m.group(1)))
    names = subprocess.run(["c++filt"], input="\n".join(n for _, n in rows), capture_output=True, text=True).stdout.split("\n")
    for (b, _), n in sorted(zip(rows, names), key=lambda x: -x[0][0]):
        print(f"{b:4d}  {n[:150]}")


if __name__ == "__main__":
    main()
