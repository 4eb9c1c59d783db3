"""torch.library registration of the sampling boundary: `skeldiff::sample_loop`.

The op is what `NonisotropicGaussianDiffusion.sample()` / `p_sample_loop` reach through
`SamplingEngine.sample_loop` (reference call stack: `base.py:439-443` -> `p_sample_loop` :343-390).
It validates shapes, dtypes and devices against the plan (`sd_plan_dims`), runs `sd_sample_loop`
on torch's current stream and raises `RuntimeError` (SkelDiffError) carrying `sd_last_error()`.
Outputs are caller-allocated and mutated in place (`out` keeps a captured hipGraph's pointers
stable across calls), so torch's dispatcher, torch.compile and graph capture see one opaque op
with declared side effects instead of a ctypes call.  A fake (meta) implementation lets the op be
traced without a device.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch
from torch import Tensor

from . import _lib
from ._lib import SkelDiffError

_side_streams = {}


def _validate(plan: int, x_cond, cond_repeat, start_noise, sampling_noise, out, noise_t, mean_t, imgs,
              start_out, workspace, flags):
    if out.dim() != 3:
        raise SkelDiffError(f"skeldiff::sample_loop: out must be (rows, J, D), got {tuple(out.shape)}")
    rows = out.shape[0]
    dims = (ctypes.c_int32 * 4)()
    _lib.check(_lib.lib().sd_plan_dims(ctypes.c_void_p(plan), dims))
    J, D, T, C = dims
    dev = out.device
    if dev.type != "cuda":
        raise SkelDiffError(f"skeldiff::sample_loop: tensors must be on a ROCm device, out is on {dev}")

    def chk(name, t, shape, optional=True, dtype=torch.float32):
        if t is None:
            if not optional:
                raise SkelDiffError(f"skeldiff::sample_loop: {name} is required")
            return
        if t.device != dev:
            raise SkelDiffError(f"skeldiff::sample_loop: {name} is on {t.device}, out on {dev}")
        if t.dtype != dtype:
            raise SkelDiffError(f"skeldiff::sample_loop: {name} must be {dtype}, got {t.dtype}")
        if not t.is_contiguous():
            raise SkelDiffError(f"skeldiff::sample_loop: {name} must be contiguous")
        if shape is not None and tuple(t.shape) != tuple(shape):
            raise SkelDiffError(f"skeldiff::sample_loop: {name} must be {tuple(shape)}, got {tuple(t.shape)}")

    tm1 = max(T - 1, 0)
    chk("out", out, (rows, J, D), optional=False)
    chk("start_noise", start_noise, (rows, J, D), optional=bool(flags & _lib.SD_FLAG_DEVICE_START))
    chk("sampling_noise", sampling_noise, (rows, tm1, J, D), optional=bool(flags & _lib.SD_FLAG_DEVICE_NOISE))
    for name, t in (("noise_t", noise_t), ("mean_t", mean_t), ("imgs", imgs)):
        chk(name, t, (rows, tm1, J, D))
    chk("start_out", start_out, (rows, J, D))
    chk("workspace", workspace, None, optional=False, dtype=torch.uint8)
    if C > 0:
        if x_cond is None:
            raise SkelDiffError("skeldiff::sample_loop: x_cond is required (diffusion_conditioning)")
        if cond_repeat < 1 or x_cond.shape[0] * cond_repeat != rows:
            raise SkelDiffError(f"skeldiff::sample_loop: x_cond rows ({x_cond.shape[0]}) x cond_repeat "
                                f"({cond_repeat}) must equal the batch ({rows}) (base.py:246-248)")
        chk("x_cond", x_cond, (x_cond.shape[0], J, C))
    return rows


@torch.library.custom_op("skeldiff::sample_loop",
                         mutates_args=("out", "noise_t", "mean_t", "imgs", "start_out", "workspace"))
def sample_loop(plan: int, x_cond: Optional[Tensor], cond_repeat: int, start_noise: Optional[Tensor],
                sampling_noise: Optional[Tensor], seed: int, row0: int, out: Tensor, noise_t: Optional[Tensor],
                mean_t: Optional[Tensor], imgs: Optional[Tensor], start_out: Optional[Tensor], workspace: Tensor,
                flags: int) -> None:
    """The reverse chain t = T-1 .. 0 (sd_sample_loop) of the plan `plan` (an sd_plan* as int)."""
    rows = _validate(plan, x_cond, cond_repeat, start_noise, sampling_noise, out, noise_t, mean_t, imgs, start_out,
                     workspace, flags)
    p = _lib.ptr
    args = (ctypes.c_void_p(plan), p(start_noise), p(x_cond), cond_repeat, p(sampling_noise), seed & (2 ** 64 - 1),
            row0, p(out), p(mean_t), p(noise_t), p(imgs), p(start_out), rows, p(workspace), workspace.numel(), flags)
    dev = out.device
    cur = torch.cuda.current_stream(dev)
    if (flags & _lib.SD_FLAG_GRAPH) and cur.cuda_stream == 0:
        # stream capture is not possible on the legacy default stream: run on a side stream
        side = _side_streams.get(dev)
        if side is None:
            side = _side_streams[dev] = torch.cuda.Stream(dev)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            _lib.check(_lib.lib().sd_sample_loop(*args, side.cuda_stream))
        cur.wait_stream(side)
        for t in (out, noise_t, mean_t, imgs, start_out, workspace):
            if t is not None:
                t.record_stream(side)
    else:
        _lib.check(_lib.lib().sd_sample_loop(*args, cur.cuda_stream))


@sample_loop.register_fake
def _(plan, x_cond, cond_repeat, start_noise, sampling_noise, seed, row0, out, noise_t, mean_t, imgs, start_out,
      workspace, flags):
    return None
