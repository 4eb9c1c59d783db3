"""Training-side StaticGraphLinear on HIP (SURVEY.md §8f "next" #4).

`GraphLinearFunction` is a torch.autograd.Function whose forward and backward are the
`sd_gl_train_forward` / `sd_gl_train_backward` kernels (include/skeldiff.h,
csrc/sd_train.hip).  It replaces, for fp32 device tensors under autograd, the einsum/matmul
forward of the reference's GraphLinear (src/core/network/layers/graph_structural.py:30-43,
StaticGraphLinear :105-114) and the backward torch derives for it when
`NonisotropicGaussianDiffusion.forward` trains the Denoiser (src/core/diffusion/base.py:262-307,
src/core/trainer.py:224-276).  The mixing matrix's own gradient flows on through torch into G
(Ghat = G / rowsum|G| is a J x J torch op).

`StaticGraphLinear.forward` (core/network/layers.py) routes here when the input is an fp32 device
tensor, grad is enabled and `hip_training_enabled()`; there is no silent CPU fallback on a GPU
(the library must load or the call raises).
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _lib

_ENABLED = True


def set_hip_training(enabled: bool) -> bool:
    """Switch the HIP training graph-linear on/off (process-wide).  Returns the previous value."""
    global _ENABLED
    prev, _ENABLED = _ENABLED, bool(enabled)
    return prev


def hip_training_enabled() -> bool:
    return _ENABLED


MAX_NODES = 64  # sd_gl_train_forward / _backward: 1 <= J <= 64


def hip_shapes_ok(x, weight, ghat, node_types) -> bool:
    """Whether a StaticGraphLinear call fits the HIP training kernels (else the torch path
    runs): J <= 64, a (J, J) mixing matrix, and a node_types vector of length J whose values
    index the weight's type axis.  Mismatches raise the torch path's own shape errors instead of
    becoming out-of-bounds device reads."""
    if x.dim() < 2:
        return False
    J = x.shape[-2]
    if not (1 <= J <= MAX_NODES) or tuple(ghat.shape) != (J, J) or weight.dim() not in (2, 3):
        return False
    if node_types is None:
        return weight.dim() == 2
    if weight.dim() != 3 or node_types.numel() != J:
        return False
    nt = node_types.detach()
    return bool((nt >= 0).all()) and int(nt.max()) < weight.shape[0]


def _stream(dev: torch.device) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


class GraphLinearFunction(torch.autograd.Function):
    """y = ghat @ (W[type j] x_j + bias[type j]) with the backward on HIP.

    x (..., J, K); weight (types, N, K) or (N, K) (shared); bias (types, N), (N,) or None;
    ghat (J, J); node_types (J,) int64 on the device or None (shared weights)."""

    @staticmethod
    def forward(ctx, x, weight, bias, ghat, node_types):
        J, K = x.shape[-2], x.shape[-1]
        lead = x.shape[:-2]
        xc = x.reshape(-1, J, K).contiguous()
        w3 = weight if weight.dim() == 3 else weight.unsqueeze(0)
        w3 = w3.contiguous()
        n_types = int(w3.shape[0]) if node_types is not None else 0
        N = int(w3.shape[1])
        if w3.shape[2] != K:
            raise ValueError(f"weight in_features {w3.shape[2]} != input features {K}")
        b2 = None if bias is None else bias.reshape(w3.shape[0], N).contiguous()
        gh = ghat.contiguous()
        nt = None if node_types is None else node_types.to(device=x.device, dtype=torch.int64).contiguous()
        rows = xc.shape[0]
        z = torch.empty(rows, J, N, device=x.device, dtype=torch.float32)
        y = torch.empty_like(z)
        _lib.check(_lib.lib().sd_gl_train_forward(
            xc.data_ptr(), w3.data_ptr(), _lib.ptr(b2), _lib.ptr(nt), n_types, gh.data_ptr(), rows, J, K, N,
            z.data_ptr(), y.data_ptr(), _stream(x.device)))
        ctx.save_for_backward(xc, z, w3, gh, nt)
        ctx.meta = (lead, J, K, N, n_types, weight.shape, None if bias is None else bias.shape)
        return y.reshape(*lead, J, N)

    @staticmethod
    def backward(ctx, dy):
        xc, z, w3, gh, nt = ctx.saved_tensors
        lead, J, K, N, n_types, wshape, bshape = ctx.meta
        need_x, need_w, need_b, need_g, _ = ctx.needs_input_grad
        dyc = dy.reshape(-1, J, N).contiguous().float()
        rows = dyc.shape[0]
        dev = dyc.device
        dx = torch.empty(rows, J, K, device=dev) if need_x else None
        dW = torch.empty(w3.shape, device=dev) if need_w else None
        db = torch.empty(w3.shape[0], N, device=dev) if (need_b and bshape is not None) else None
        dg = torch.empty(J, J, device=dev) if need_g else None
        L = _lib.lib()
        ws_bytes = L.sd_gl_train_workspace_bytes(rows, J, K, N, n_types)
        ws = torch.empty((ws_bytes + 3) // 4, device=dev, dtype=torch.float32)
        _lib.check(L.sd_gl_train_backward(
            xc.data_ptr(), z.data_ptr(), dyc.data_ptr(), w3.data_ptr(), _lib.ptr(nt), n_types, gh.data_ptr(), rows,
            J, K, N, _lib.ptr(dx), _lib.ptr(dW), _lib.ptr(db), _lib.ptr(dg), ws.data_ptr(), ws_bytes, _stream(dev)))
        return (None if dx is None else dx.reshape(*lead, J, K),
                None if dW is None else dW.reshape(wshape),
                None if db is None else db.reshape(bshape),
                dg, None)


class AttentionCoreFunction(torch.autograd.Function):
    """out = softmax((q scale) k^T) v per head over the joint axis, from to_qkv's output
    (reference attention.py:122-136, without dropout / q-k norms), forward and backward on HIP
    (`sd_attn_train_forward` / `_backward`, csrc/sd_train.hip).  qkv (..., J, 3 * heads * dim_head)
    -> (..., J, heads * dim_head)."""

    @staticmethod
    def forward(ctx, qkv, heads: int, dim_head: int, scale: float):
        J, W = qkv.shape[-2], qkv.shape[-1]
        if W != 3 * heads * dim_head:
            raise ValueError(f"qkv width {W} != 3 * {heads} * {dim_head}")
        lead = qkv.shape[:-2]
        qc = qkv.reshape(-1, J, W).contiguous()
        rows = qc.shape[0]
        out = torch.empty(rows, J, heads * dim_head, device=qkv.device, dtype=torch.float32)
        _lib.check(_lib.lib().sd_attn_train_forward(qc.data_ptr(), out.data_ptr(), rows, J, heads, dim_head,
                                                     float(scale), _stream(qkv.device)))
        ctx.save_for_backward(qc)
        ctx.meta = (lead, J, heads, dim_head, float(scale))
        return out.reshape(*lead, J, heads * dim_head)

    @staticmethod
    def backward(ctx, dout):
        (qc,) = ctx.saved_tensors
        lead, J, heads, dim_head, scale = ctx.meta
        dc = dout.reshape(-1, J, heads * dim_head).contiguous().float()
        dqkv = torch.empty_like(qc)
        _lib.check(_lib.lib().sd_attn_train_backward(qc.data_ptr(), dc.data_ptr(), dqkv.data_ptr(), qc.shape[0], J,
                                                      heads, dim_head, scale, _stream(qc.device)))
        return dqkv.reshape(*lead, J, 3 * heads * dim_head), None, None, None


def attention_core(qkv: torch.Tensor, heads: int, dim_head: int, scale: float) -> torch.Tensor:
    """HIP attention core under autograd (fp32 device tensors, J <= 64, dim_head <= 64)."""
    if not qkv.is_cuda or qkv.dtype != torch.float32:
        raise ValueError("attention_core: the HIP training path needs fp32 device tensors")
    return AttentionCoreFunction.apply(qkv, heads, dim_head, scale)


class FilmTanhFunction(torch.autograd.Function):
    """tanh(y (scale + 1) + shift) with (scale | shift) = ss (rows, 1, 2C) broadcast over the J
    nodes -- a ResnetBlock's first Block after its graph-linear (reference attention.py:67-75) --
    forward and backward on HIP (`sd_film_tanh_forward` / `_backward`)."""

    @staticmethod
    def forward(ctx, y, ss):
        rows, J, C = y.shape
        yc = y.contiguous()
        sc = ss.reshape(rows, 2 * C).contiguous()
        out = torch.empty_like(yc)
        _lib.check(_lib.lib().sd_film_tanh_forward(yc.data_ptr(), sc.data_ptr(), out.data_ptr(), rows, J, C,
                                                    _stream(y.device)))
        ctx.save_for_backward(yc, sc, out)
        ctx.ss_shape = ss.shape
        return out

    @staticmethod
    def backward(ctx, dout):
        yc, sc, out = ctx.saved_tensors
        rows, J, C = yc.shape
        dc = dout.contiguous().float()
        dy = torch.empty_like(yc)
        dss = torch.empty_like(sc)
        _lib.check(_lib.lib().sd_film_tanh_backward(yc.data_ptr(), sc.data_ptr(), out.data_ptr(), dc.data_ptr(),
                                                     dy.data_ptr(), dss.data_ptr(), rows, J, C, _stream(yc.device)))
        return dy, dss.reshape(ctx.ss_shape)


def film_tanh(y: torch.Tensor, ss: torch.Tensor) -> torch.Tensor:
    """HIP FiLM + tanh under autograd: y (rows, J, C) fp32 on the device, ss (rows, 1, 2C)."""
    if not y.is_cuda or y.dtype != torch.float32 or ss.dtype != torch.float32:
        raise ValueError("film_tanh: the HIP training path needs fp32 device tensors")
    return FilmTanhFunction.apply(y, ss)


def graph_linear(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor], ghat: torch.Tensor,
                 node_types: Optional[torch.Tensor]) -> torch.Tensor:
    """HIP StaticGraphLinear under autograd (fp32 device tensors)."""
    if not x.is_cuda:
        raise ValueError("graph_linear: the HIP training path needs device tensors")
    if x.dtype != torch.float32 or weight.dtype != torch.float32:
        raise ValueError("graph_linear: the HIP training path is fp32")
    return GraphLinearFunction.apply(x, weight, bias, ghat, node_types)
