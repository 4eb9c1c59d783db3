"""The torch.library boundary op skeldiff::sample_loop (skeletondiffusion_amd/ops.py):
registered with its schema and side effects, traceable without a device (fake impl), and
validating on the host -- shapes against the plan's dims (sd_plan_dims), dtypes and devices --
with RuntimeError (SkelDiffError) before any device work.  The GPU path is exercised by every
sample() in the -m gpu suite (engine.sample_loop calls the op) and by test_op_direct_call."""
import ctypes
import re

import pytest
import torch

from skeletondiffusion_amd import _lib, ops  # noqa: F401
from skeletondiffusion_amd._lib import SkelDiffError


def test_op_registered_with_mutation_schema():
    schema = str(torch.ops.skeldiff.sample_loop.default._schema)
    assert schema.startswith("skeldiff::sample_loop(")
    for name in ("out", "noise_t", "mean_t", "imgs", "start_out", "workspace"):
        assert re.search(rf"Tensor\(a\d+!\)\??\s+{name}\b", schema), (name, schema)


def _plan(J=16, D=96, T=10, cond=96):
    d = _lib.SDPlanDesc(num_nodes=J, latent_dim=D, cond_dim=cond, out_dim=D, depth=1, attn_heads=4, attn_dim_head=32,
                        use_attention=1, self_condition=0, learn_influence=0, num_node_types=0, timesteps=T,
                        isotropic=0, activation=0, sinusoidal_theta=10000.0)
    h = ctypes.c_void_p()
    assert _lib.lib().sd_plan_create(ctypes.byref(h), ctypes.byref(d)) == 0
    return h


def test_plan_dims():
    h = _plan(J=17, D=96, T=100, cond=96)
    try:
        dims = (ctypes.c_int32 * 4)()
        assert _lib.lib().sd_plan_dims(h, dims) == 0
        assert list(dims) == [17, 96, 100, 96]
    finally:
        _lib.lib().sd_plan_destroy(h)


def test_op_validates_on_host():
    """CPU tensors are refused before any library call that touches a device; so are wrong
    shapes (checked against the plan) -- RuntimeError subclasses carrying the reason."""
    h = _plan()
    try:
        out = torch.empty((8, 16, 96))
        ws = torch.empty(16, dtype=torch.uint8)
        flags = _lib.SD_FLAG_DEVICE_START | _lib.SD_FLAG_DEVICE_NOISE
        with pytest.raises(RuntimeError, match="ROCm device"):
            torch.ops.skeldiff.sample_loop(h.value, None, 1, None, None, 1, 0, out, None, None, None, None, ws, flags)
        with pytest.raises(SkelDiffError, match=r"out must be \(rows, J, D\)"):
            torch.ops.skeldiff.sample_loop(h.value, None, 1, None, None, 1, 0, torch.empty(8, 16), None, None, None,
                                           None, ws, flags)
    finally:
        _lib.lib().sd_plan_destroy(h)


def test_op_traces_with_fake_tensors():
    """The fake implementation: the op can be traced (meta tensors, no device, no library call)."""
    from torch._subclasses.fake_tensor import FakeTensorMode

    with FakeTensorMode():
        out = torch.empty((8, 16, 96))
        ws = torch.empty(16, dtype=torch.uint8)
        assert torch.ops.skeldiff.sample_loop(0, None, 1, None, None, 1, 0, out, None, None, None, None, ws, 6) is None
