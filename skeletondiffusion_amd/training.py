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


class L1NormRowsFunction(torch.autograd.Function):
    """Ghat_k = G_k / max(rowsum|G_k|, eps) (F.normalize(G, p=1, dim=1), reference
    graph_structural.py:107) for L matrices G_1 .. G_L of one size, forward and backward on HIP
    (`sd_l1norm_rows_forward` / `_backward`, one launch each way for all L): the Denoiser
    normalises all its learnable G at once per forward instead of torch's norm / clamp / div chain
    and its backward per StaticGraphLinear call.  apply(eps, G_1, ..., G_L) -> (Ghat_1, ..., Ghat_L)."""

    @staticmethod
    def forward(ctx, eps: float, *Gs):
        Gc = torch.stack([g.detach() for g in Gs]).contiguous()
        L, J = Gc.shape[0], Gc.shape[1]
        out = torch.empty_like(Gc)
        _lib.check(_lib.lib().sd_l1norm_rows_forward(Gc.data_ptr(), out.data_ptr(), J, L, float(eps),
                                                      _stream(Gc.device)))
        ctx.save_for_backward(Gc)
        ctx.eps = float(eps)
        return tuple(out.unbind(0))

    @staticmethod
    def backward(ctx, *douts):
        (Gc,) = ctx.saved_tensors
        L, J = Gc.shape[0], Gc.shape[1]
        dc = torch.stack([torch.zeros_like(Gc[0]) if d is None else d.float() for d in douts]).contiguous()
        dG = torch.empty_like(Gc)
        _lib.check(_lib.lib().sd_l1norm_rows_backward(Gc.data_ptr(), dc.data_ptr(), dG.data_ptr(), J, L, ctx.eps,
                                                       _stream(Gc.device)))
        return (None,) + tuple(dG.unbind(0))


def l1norm_rows_many(Gs, eps: float = 1e-12):
    """HIP row-wise L1 normalisation of L (J, J) fp32 device matrices under autograd (J <= 64), one
    launch each way."""
    Gs = list(Gs)
    if not Gs:
        return ()
    J = Gs[0].shape[0]
    for G in Gs:
        if (not G.is_cuda or G.dtype != torch.float32 or G.dim() != 2 or tuple(G.shape) != (J, J)
                or J > MAX_NODES or G.device != Gs[0].device):
            raise ValueError("l1norm_rows: the HIP training path needs (J, J) fp32 device matrices, J <= 64")
    return L1NormRowsFunction.apply(eps, *Gs)


def l1norm_rows(G: torch.Tensor, eps: float = 1e-12) -> torch.Tensor:
    """HIP row-wise L1 normalisation of one (J, J) fp32 device matrix under autograd (J <= 64)."""
    return l1norm_rows_many([G], eps)[0]


class RMSNormFunction(torch.autograd.Function):
    """PreNorm's RMSNorm, x / max(||x||, eps) * g * sqrt(C) over the last axis (reference
    attention.py:30-36), forward and backward on HIP (`sd_rmsnorm_forward` / `_backward`)."""

    @staticmethod
    def forward(ctx, x, g, scale: float, eps: float):
        C = x.shape[-1]
        xc = x.reshape(-1, C).contiguous()
        gc = g.reshape(C).contiguous()
        R = xc.shape[0]
        out = torch.empty_like(xc)
        dnorm = torch.empty(R, device=x.device, dtype=torch.float32)
        _lib.check(_lib.lib().sd_rmsnorm_forward(xc.data_ptr(), gc.data_ptr(), out.data_ptr(), dnorm.data_ptr(), R, C,
                                                  float(scale), float(eps), _stream(x.device)))
        ctx.save_for_backward(xc, gc, dnorm)
        ctx.meta = (x.shape, g.shape, float(scale), float(eps))
        return out.reshape(x.shape)

    @staticmethod
    def backward(ctx, dout):
        xc, gc, dnorm = ctx.saved_tensors
        xshape, gshape, scale, eps = ctx.meta
        R, C = xc.shape
        dc = dout.reshape(R, C).contiguous().float()
        dx = torch.empty_like(xc)
        dg = torch.empty(C, device=xc.device, dtype=torch.float32)
        L = _lib.lib()
        ws_bytes = L.sd_rmsnorm_workspace_bytes(R, C)
        ws = torch.empty(max(1, (ws_bytes + 3) // 4), device=xc.device, dtype=torch.float32)
        _lib.check(L.sd_rmsnorm_backward(xc.data_ptr(), gc.data_ptr(), dnorm.data_ptr(), dc.data_ptr(), dx.data_ptr(),
                                         dg.data_ptr(), R, C, scale, eps, ws.data_ptr(), ws_bytes, _stream(xc.device)))
        return dx.reshape(xshape), dg.reshape(gshape), None, None


def rmsnorm(x: torch.Tensor, g: torch.Tensor, scale: float, eps: float = 1e-12) -> torch.Tensor:
    """HIP RMSNorm under autograd: x (..., C) and g (C elements) fp32 on the device, C <= 1024."""
    if not x.is_cuda or x.dtype != torch.float32 or g.dtype != torch.float32 or x.shape[-1] > 1024:
        raise ValueError("rmsnorm: the HIP training path needs fp32 device tensors with C <= 1024")
    return RMSNormFunction.apply(x, g, scale, eps)


class MahalanobisLossFunction(torch.autograd.Function):
    """Per-row Mahalanobis loss of NonisotropicGaussianDiffusion: mean over (J, F) of
    |S[t] D| (l1) or (S[t] D)^2 (mse), D = target - model_out (pred_noise) or model_out - target
    (reference nonisotropic.py:177-190 + the 'b ... -> b' mean of base.py:298), forward and
    backward on HIP (`sd_mahalanobis_loss_forward` / `_backward`).  The target gets the negated
    gradient of model_out."""

    @staticmethod
    def forward(ctx, model_out, target, S, t, pred_noise: bool, mse: bool):
        rows, J, F = model_out.shape
        mo = model_out.contiguous()
        tg = target.contiguous().float()
        Sc = S.contiguous()
        tc = t.to(device=mo.device, dtype=torch.int64).contiguous()
        loss = torch.empty(rows, device=mo.device, dtype=torch.float32)
        _lib.check(_lib.lib().sd_mahalanobis_loss_forward(mo.data_ptr(), tg.data_ptr(), Sc.data_ptr(), tc.data_ptr(),
                                                           Sc.shape[0], rows, J, F, int(pred_noise), int(mse), loss.data_ptr(),
                                                           _stream(mo.device)))
        ctx.save_for_backward(mo, tg, Sc, tc)
        ctx.flags = (int(pred_noise), int(mse))
        return loss

    @staticmethod
    def backward(ctx, dloss):
        mo, tg, Sc, tc = ctx.saved_tensors
        pred_noise, mse = ctx.flags
        rows, J, F = mo.shape
        dl = dloss.contiguous().float()
        dmo = torch.empty_like(mo)
        _lib.check(_lib.lib().sd_mahalanobis_loss_backward(mo.data_ptr(), tg.data_ptr(), Sc.data_ptr(), tc.data_ptr(),
                                                            Sc.shape[0], dl.data_ptr(), rows, J, F, pred_noise, mse, dmo.data_ptr(),
                                                            _stream(mo.device)))
        need_mo, need_tg = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        return (dmo if need_mo else None), (-dmo if need_tg else None), None, None, None, None


def mahalanobis_loss(model_out: torch.Tensor, target: torch.Tensor, S: torch.Tensor, t: torch.Tensor,
                     pred_noise: bool, mse: bool) -> torch.Tensor:
    """HIP per-row Mahalanobis loss under autograd: model_out / target (rows, J, F) fp32 on the
    device, S (T, J, J), t (rows,) timesteps; J <= 64, F <= 256."""
    if (not model_out.is_cuda or model_out.dtype != torch.float32 or model_out.dim() != 3
            or model_out.shape[1] > MAX_NODES or model_out.shape[2] > 256 or S.dtype != torch.float32):
        raise ValueError("mahalanobis_loss: the HIP training path needs (rows, J <= 64, F <= 256) fp32 device tensors")
    return MahalanobisLossFunction.apply(model_out, target, S, t, pred_noise, mse)


# ---- best-of-k training relaxation (reference src/core/trainer.py:182-222) -----

class BestOfKFunction(torch.autograd.Function):
    """Per sequence the sample whose similarity is smallest and the diffusion loss there:
    `loss_similarity.view(b, -1).min(axis=-1).indices` + `torch.gather` of get_ksimilarity_loss
    (trainer.py:207-222), forward and backward on HIP (`sd_best_of_k` / `_backward`).  The
    similarity carries no gradient (the reference computes it under no_grad)."""

    @staticmethod
    def forward(ctx, loss, sim, k: int):
        lv = loss.contiguous().view(-1)
        nseq = lv.numel() // k
        sv = None if sim is None else sim.detach().contiguous().float().view(-1)
        idx = torch.empty(nseq, device=lv.device, dtype=torch.int64)
        sel = torch.empty(nseq, device=lv.device, dtype=torch.float32)
        _lib.check(_lib.lib().sd_best_of_k(None if sv is None else sv.data_ptr(), lv.data_ptr(), nseq, k,
                                           idx.data_ptr(), sel.data_ptr(), _stream(lv.device)))
        ctx.save_for_backward(idx)
        ctx.k = k
        ctx.mark_non_differentiable(idx)
        return sel, idx

    @staticmethod
    def backward(ctx, dsel, _didx):
        (idx,) = ctx.saved_tensors
        k = ctx.k
        nseq = idx.numel()
        dl = torch.empty(nseq * k, device=idx.device, dtype=torch.float32)
        ds = dsel.contiguous().float()
        _lib.check(_lib.lib().sd_best_of_k_backward(ds.data_ptr(), idx.data_ptr(), nseq, k, dl.data_ptr(),
                                                    _stream(idx.device)))
        return dl, None, None


def best_of_k(loss: torch.Tensor, k: int, sim: Optional[torch.Tensor] = None):
    """(nseq * k,) per-sample diffusion losses (sequence-major: p_losses' repeat_interleave order,
    base.py:264-268) -> (selected loss (nseq,), index (nseq,)): the sample with the smallest `sim`
    (nseq * k values; default the loss itself: the latent space) per sequence, as
    get_ksimilarity_loss (trainer.py:207-222)."""
    if not loss.is_cuda or loss.dtype != torch.float32 or loss.numel() % k or k < 1:
        raise ValueError("best_of_k: an fp32 device tensor of nseq * k losses is required")
    if sim is not None and (sim.numel() != loss.numel() or sim.device != loss.device):
        raise ValueError("best_of_k: sim must hold one value per loss, on the same device")
    return BestOfKFunction.apply(loss, sim, int(k))


def pose_loss(pred: torch.Tensor, target: torch.Tensor, mse: bool) -> torch.Tensor:
    """AutoEncoder.loss(pred, target, reduction='none') (autoencoder.py:80-98) on HIP (`sd_pose_loss`),
    no grad: pred (nseq, S, T, J, C), target (nseq, T, J, C) -> (nseq, S)."""
    if not pred.is_cuda or pred.dim() != 5 or target.dim() != 4 or pred.shape[0] != target.shape[0] or \
            tuple(pred.shape[2:]) != tuple(target.shape[1:]):
        raise ValueError("pose_loss: pred (nseq, S, T, J, C) and target (nseq, T, J, C) device tensors")
    nseq, S, T, J, C = pred.shape
    p = pred.detach().contiguous().float()
    tg = target.detach().contiguous().float()
    out = torch.empty((nseq, S), device=pred.device, dtype=torch.float32)
    _lib.check(_lib.lib().sd_pose_loss(p.data_ptr(), tg.data_ptr(), nseq, S, T, J, C, int(bool(mse)), out.data_ptr(),
                                       _stream(pred.device)))
    return out
