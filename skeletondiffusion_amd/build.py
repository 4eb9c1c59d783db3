"""In-tree build of libskeldiff.so with hipcc for gfx950 (no torch extension machinery: the
library exposes a plain C ABI, include/skeldiff.h)."""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libskeldiff.so")
SOURCES = ["sd_kernels.hip", "sd_graph_linear.hip", "sd_graph_linear_v3.hip", "sd_graph_linear_v4.hip", "sd_graph_linear_v5.hip",
           "sd_metrics.hip", "sd_decoder.hip", "sd_train.hip", "sd_plan.hip"]
HEADERS = ["sd_internal.h", os.path.join("..", "..", "include", "skeldiff.h")]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def _stale(stamp: str) -> bool:
    """The product library is rebuilt when a source is newer or it was built with other flags
    (the stamp beside it records them: a diagnostic build can never pass for the product)."""
    if not os.path.exists(OUT) or not os.path.exists(OUT + ".flags"):
        return True
    with open(OUT + ".flags") as f:
        if f.read() != stamp:
            return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(os.path.join(CSRC, f)) > t for f in SOURCES + HEADERS)


# Device code is compiled WITHOUT packed-FP32 instructions (v_pk_fma/mul/add_f32).  Measured on
# MI355X: a packed-FP32 instruction reading a register just written by an LDS load
# returned zeros in lanes 48-63 whenever a workgroup of another kernel shared the CU (row chains,
# concurrent plans), so the posterior update drew sigma * eps = 0 for some latents; with the
# feature off every row-chain configuration is bitwise equal to one chain, at unchanged speed.
# (The host pass of each hipcc call ignores the feature, with a one-line note that build filters.)
DEVICE_FLAGS = ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]
_FEATURE_NOTE = b"'-packed-fp32-ops' is not a recognized feature for this target"


def build_library(force: bool = False, verbose: bool = False, debug_lds: bool = False, extra=(), tag="_dbg",
                  packed_fp32: bool = False) -> str:
    """debug_lds: the diagnostic variant libskeldiff_dbg.so (-DSD_DEBUG_LDS: LDS integrity
    counters in k_gl4 / k_update, sd_debug_lds_counters); load it with SKELDIFF_LIB.
    packed_fp32: the round-3 hazard reproduction build, always a tagged
    diagnostic variant (libskeldiff_packed.so unless `tag` says otherwise).
    Every product build is checked after linking (isa_check: gfx950 code objects only, no
    packed-FP32 instruction) and stamped with its flags."""
    variant = debug_lds or bool(extra) or packed_fp32  # a diagnostic variant: libskeldiff{tag}.so, never the product
    if packed_fp32 and tag == "_dbg":
        tag = "_packed"
    out = OUT.replace(".so", tag + ".so") if variant else OUT
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wno-pass-failed"] + \
        ([] if packed_fp32 else DEVICE_FLAGS) + (["-DSD_DEBUG_LDS"] if debug_lds else []) + list(extra)
    stamp = " ".join(flags)
    if not force and not variant and not _stale(stamp):
        return OUT
    info = "no-packed-fp32" if not packed_fp32 else "packed-fp32 (diagnostic)"
    objs, procs = [], []
    for src in SOURCES:  # one hipcc per translation unit, in parallel
        obj = os.path.join(CSRC, src.replace(".hip", tag + ".o" if variant else ".o"))
        cmd = [_hipcc(), "-c"] + flags + [f'-DSD_BUILD_INFO="{info}"', os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append((src, subprocess.Popen(cmd, stderr=subprocess.PIPE)))
        objs.append(obj)
    failed = []
    for src, pr in procs:
        _, err = pr.communicate()
        msg = b"\n".join(l for l in err.splitlines() if _FEATURE_NOTE not in l)
        if msg.strip():
            sys.stderr.write(msg.decode(errors="replace") + "\n")
        if pr.returncode != 0:
            failed.append(src)
    if failed:
        raise RuntimeError("hipcc failed: " + ", ".join(failed))
    tmp = out + ".tmp"
    subprocess.run([_hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", tmp] + objs, check=True)
    for o in objs:
        os.remove(o)
    if not variant:
        try:
            from . import isa_check
        except ImportError:  # run as a script
            import isa_check
        try:
            isa_check.check(tmp)  # a packed-FP32 or non-gfx950 build never becomes the product
        except Exception:
            os.remove(tmp)
            raise
    os.replace(tmp, out)
    if not variant:
        with open(OUT + ".flags", "w") as f:
            f.write(stamp)
    return out


if __name__ == "__main__":
    print(build_library(force=True, verbose=True, debug_lds="--debug-lds" in sys.argv))
