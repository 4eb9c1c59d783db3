"""Instruction-class guard for the built library.

Rows were computed wrong whenever a packed-FP32 VOP3P instruction (v_pk_fma_f32 / v_pk_mul_f32 /
v_pk_add_f32) ran while a workgroup of another kernel shared the CU; the library is therefore
compiled without the packed-FP32 target feature (build.py).  This module proves that on the
binary itself: it splits the `.hip_fatbin` section of libskeldiff.so into its clang offload
bundles, takes every device code object, disassembles it for gfx950 and counts the packed-FP32
instructions (must be 0), the MFMA instructions (a sanity floor: the kernels are MFMA code) and the
targets (gfx950 only).  build.build_library() runs it after every product link, and
tests/test_isa_guard.py runs it on the shipped library.
"""
from __future__ import annotations

import os
import re
import struct
import subprocess
import tempfile

LLVM_BIN = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
PACKED_F32 = re.compile(r"\bv_pk_(fma|mul|add)_f32\b")
MFMA = re.compile(r"\bv_mfma_\w+")


def _tool(name: str) -> str:
    p = os.path.join(LLVM_BIN, name)
    if not os.path.exists(p):
        raise RuntimeError(f"{p} not found (ROCm LLVM tools)")
    return p


def fatbin_section(so_path: str) -> bytes:
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "fatbin")
        subprocess.run([_tool("llvm-objcopy"), "--dump-section", f".hip_fatbin={out}", so_path, os.path.join(td, "x")],
                       check=True, capture_output=True)
        with open(out, "rb") as f:
            return f.read()


def code_objects(so_path: str):
    """[(target triple, code object bytes)] of every offload bundle in the library's fatbin."""
    data = fatbin_section(so_path)
    objs = []
    pos = data.find(MAGIC)
    while pos >= 0:
        (n,) = struct.unpack_from("<Q", data, pos + len(MAGIC))
        q = pos + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, q)
            triple = data[q + 24:q + 24 + tlen].decode()
            q += 24 + tlen
            if size and triple.startswith("hip"):
                objs.append((triple, data[pos + off:pos + off + size]))
        pos = data.find(MAGIC, pos + len(MAGIC))
    return objs


def scan(so_path: str) -> dict:
    """Disassemble every device code object: {'targets': set, 'objects': n, 'packed_f32': {op: n},
    'mfma': n}."""
    res = {"targets": set(), "objects": 0, "packed_f32": {}, "mfma": 0}
    with tempfile.TemporaryDirectory() as td:
        for i, (triple, blob) in enumerate(code_objects(so_path)):
            res["targets"].add(triple.rsplit("-", 1)[-1])
            path = os.path.join(td, f"co{i}.o")
            with open(path, "wb") as f:
                f.write(blob)
            asm = subprocess.run([_tool("llvm-objdump"), "-d", "--mcpu=gfx950", path], check=True,
                                 capture_output=True, text=True).stdout
            res["objects"] += 1
            for m in PACKED_F32.finditer(asm):
                op = m.group(0)
                res["packed_f32"][op] = res["packed_f32"].get(op, 0) + 1
            res["mfma"] += len(MFMA.findall(asm))
    return res


# kernel-level keys of amdhsa.kernels: a kernel's map starts with "  - ." and its own keys sit at
# 4 columns (its .args entries deeper)
_NOTE_KEY = re.compile(r"^(  - |    )\.(name|vgpr_count|agpr_count|sgpr_count|private_segment_fixed_size|"
                       r"group_segment_fixed_size|vgpr_spill_count|sgpr_spill_count):\s*(\S+)\s*$")


def resources(so_path: str) -> dict:
    """{kernel symbol: {'vgpr_count', 'agpr_count', 'sgpr_count', 'private_segment_fixed_size'
    (scratch bytes per lane), 'group_segment_fixed_size' (static LDS), 'vgpr_spill_count', ...}}
    from the AMDGPU metadata notes of every device code object (`llvm-readelf --notes`)."""
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for i, (_, blob) in enumerate(code_objects(so_path)):
            path = os.path.join(td, f"co{i}.o")
            with open(path, "wb") as f:
                f.write(blob)
            notes = subprocess.run([_tool("llvm-readelf"), "--notes", path], check=True, capture_output=True,
                                   text=True).stdout
            cur = {}
            for line in notes.splitlines():
                if line.startswith("  - "):  # a new kernel's map begins
                    if ".name" in cur:
                        out[cur.pop(".name")] = cur
                    cur = {}
                m = _NOTE_KEY.match(line)
                if m:
                    _, k, v = m.groups()
                    cur["." + k if k == "name" else k] = v if k == "name" else int(v)
            if ".name" in cur:
                out[cur.pop(".name")] = cur
    return out


def check(so_path: str) -> dict:
    """Raise RuntimeError unless every code object is gfx950 code without packed-FP32 instructions."""
    r = scan(so_path)
    problems = []
    if r["objects"] == 0:
        problems.append("no device code objects found")
    if r["targets"] != {"gfx950"}:
        problems.append(f"targets {sorted(r['targets'])} (want gfx950 only)")
    if r["packed_f32"]:
        problems.append(f"packed-FP32 instructions present: {r['packed_f32']}")
    if r["mfma"] < 1000:
        problems.append(f"only {r['mfma']} MFMA instructions (not the engine's kernels?)")
    if problems:
        raise RuntimeError(f"{so_path}: " + "; ".join(problems))
    return r


if __name__ == "__main__":
    import sys

    print(check(sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "libskeldiff.so")))
