"""CPU guard of the round-3 hazard fix: the shipped libskeldiff.so holds gfx950
code objects only, none of them contains a packed-FP32 instruction (v_pk_fma_f32 / v_pk_mul_f32 /
v_pk_add_f32, the class that returned zeros beside another kernel's workgroup on a shared CU), and
the library reports the product build.  The scanner itself is checked on a small library built
here WITH packed FP32, so a silent scanner cannot pass the guard.  build.build_library() runs the
same check after every product link."""
import os
import shutil
import subprocess

import pytest

from conftest import REPO
from skeletondiffusion_amd import _lib, isa_check

LIB = os.path.join(REPO, "skeletondiffusion_amd", "libskeldiff.so")


def test_shipped_library_has_no_packed_fp32():
    r = isa_check.scan(LIB)
    assert r["targets"] == {"gfx950"}, r["targets"]
    assert r["objects"] >= 8, r["objects"]  # one per translation unit with kernels
    assert r["packed_f32"] == {}, r["packed_f32"]
    assert r["mfma"] > 10_000, r["mfma"]
    isa_check.check(LIB)


def test_library_reports_product_build():
    assert _lib.lib().sd_build_info() == b"no-packed-fp32"


def test_product_build_is_stamped_with_its_flags():
    from skeletondiffusion_amd import build

    with open(build.OUT + ".flags") as f:
        stamp = f.read()
    assert "-packed-fp32-ops" in stamp and "--offload-arch=gfx950" in stamp


KERNEL = r"""
#include <hip/hip_runtime.h>
typedef float f2 __attribute__((ext_vector_type(2)));
__global__ void k(f2* a, const f2* b, const f2* c, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = a[i] * b[i] + c[i] * b[i] + a[i];
}
"""


@pytest.mark.skipif(not shutil.which("hipcc") and not os.path.exists("/opt/rocm/bin/hipcc"), reason="no hipcc")
def test_scanner_finds_packed_fp32(tmp_path):
    """A library compiled with the default target features (packed FP32 allowed) is flagged, and
    the same source built with build.py's device flags is clean."""
    from skeletondiffusion_amd import build

    src = tmp_path / "k.hip"
    src.write_text(KERNEL)
    hipcc = build._hipcc()
    bad = tmp_path / "libbad.so"
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", str(src), "-o", str(bad)], check=True,
                   capture_output=True)
    r = isa_check.scan(str(bad))
    assert r["targets"] == {"gfx950"} and sum(r["packed_f32"].values()) > 0, r
    with pytest.raises(RuntimeError, match="packed-FP32"):
        isa_check.check(str(bad))
    good = tmp_path / "libgood.so"
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-fPIC", "-shared"] + build.DEVICE_FLAGS +
                   [str(src), "-o", str(good)], check=True, capture_output=True)
    assert isa_check.scan(str(good))["packed_f32"] == {}
