"""On-device evaluation metrics with the reference's signatures (src/metrics/multimodal.py),
computed by libskeldiff (sd_pairwise_distances / sd_ade_fde) where the sampled latents or the
decoded motions already live.  Inputs must be ROCm tensors (no CPU path); results are float32
tensors on the same device, one value per sequence (or per (sequence, sample) for
reduction != 'mean'), reduced in a fixed order (deterministic).

    lat_apd(lat_pred)                 multimodal.py:137-151  mean pairwise L1 over samples
    apd(pred, t0=0, t=-1)             multimodal.py:15-35    mean pairwise L2 over samples
    ade(target, pred, t0, t, reduction)  multimodal.py:44-57  min over samples of mean-frame L2
    fde(target, pred, t0, t, reduction)  multimodal.py:60-73  min over samples of last-frame L2

Up to 64 samples per sequence (the release evaluation draws 50).
"""
from __future__ import annotations

import torch

from . import _lib
from ._lib import SkelDiffError, check


def _device_tensor(x: torch.Tensor, name: str) -> torch.Tensor:
    if not torch.is_tensor(x) or x.device.type != "cuda":
        raise SkelDiffError(f"{name}: metrics run on the MI355X HIP engine only; pass a ROCm tensor")
    return x.detach().to(torch.float32).contiguous()


def _time_slice(x: torch.Tensor, t0: int, t: int, axis: int) -> torch.Tensor:
    """multimodal.py:4-8: frames [t0, t) of `axis`, or [t0, end) for t == -1."""
    end = x.shape[axis] if t == -1 else t
    return x.narrow(axis, t0, end - t0)


def _flat(shape) -> int:
    n = 1
    for s in shape:
        n *= int(s)
    return n


def _pairwise(x: torch.Tensor, want_l1: bool) -> torch.Tensor:
    B, S = x.shape[:2]
    x = _device_tensor(x.reshape(B, S, _flat(x.shape[2:])), "pairwise")
    out = torch.empty(B, device=x.device, dtype=torch.float32)
    l1 = out if want_l1 else None
    l2 = None if want_l1 else out
    stream = torch.cuda.current_stream(x.device).cuda_stream
    check(_lib.lib().sd_pairwise_distances(x.data_ptr(), B, S, x.shape[2], _lib.ptr(l1), _lib.ptr(l2), stream))
    return out


def lat_apd(lat_pred: torch.Tensor, **kwargs) -> torch.Tensor:
    """Average pairwise L1 distance between the samples in latent space; lat_pred
    (batch, num_samples, ...) -> (batch,)."""
    return _pairwise(lat_pred, True)


def apd(pred: torch.Tensor, t0: int = 0, t: int = -1, **kwargs) -> torch.Tensor:
    """Average pairwise L2 distance; pred (batch, num_samples, seq_length, ...) -> (batch,)."""
    pred = _time_slice(pred, t0, t, 2)
    B, S = pred.shape[:2]
    if S == 1:  # multimodal.py:19-20
        return torch.tensor([0] * B, device=pred.device)
    return _pairwise(pred, False)


def _ade_fde(target, pred, t0, t, reduction, want_ade):
    pred, target = _time_slice(pred, t0, t, 2), _time_slice(target, t0, t, 1)
    B, S, T = pred.shape[:3]
    p = _device_tensor(pred.reshape(B, S, T, _flat(pred.shape[3:])), "pred")
    g = _device_tensor(target.reshape(B, T, _flat(target.shape[2:])), "target")
    if g.shape[2] != p.shape[3]:
        raise ValueError(f"target frames have {g.shape[2]} features, pred frames {p.shape[3]}")
    dev = p.device
    best = torch.empty(B, device=dev, dtype=torch.float32)
    per = torch.empty(B, S, device=dev, dtype=torch.float32) if reduction != "mean" else None
    stream = torch.cuda.current_stream(dev).cuda_stream
    args = (best, None, per, None) if want_ade else (None, best, None, per)
    check(_lib.lib().sd_ade_fde(p.data_ptr(), g.data_ptr(), B, S, T, p.shape[3], *(_lib.ptr(a) for a in args), stream))
    return best if reduction == "mean" else per


def ade(target: torch.Tensor, pred: torch.Tensor, t0: int = 0, t: int = -1, reduction: str = "mean", **kwargs):
    """target (batch, seq_length, ...), pred (batch, num_samples, seq_length, ...): min over samples
    of the mean over frames of the L2 distance (reduction 'mean'), else the (batch, num_samples)
    distances."""
    return _ade_fde(target, pred, t0, t, reduction, True)


def fde(target: torch.Tensor, pred: torch.Tensor, t0: int = 0, t: int = -1, reduction: str = "mean", **kwargs):
    """As ade, on the last frame of the slice only."""
    return _ade_fde(target, pred, t0, t, reduction, False)


def _mm(target, pred, mm_gt, t0, t, want_ade):
    pred = _time_slice(pred, t0, t, 2)
    B, S, T = pred.shape[:3]
    if len(mm_gt) != B:
        raise ValueError(f"mm_gt has {len(mm_gt)} entries for {B} sequences")
    p = _device_tensor(pred.reshape(B, S, T, _flat(pred.shape[3:])), "pred")
    dev, F = p.device, p.shape[3]
    counts = [int(g.shape[0]) for g in mm_gt]
    if min(counts, default=1) == 0:  # the reference's reshape of an empty set raises (multimodal.py:113)
        raise RuntimeError("mmade/mmfde: a sequence has no multimodal ground truths")
    parts = [_time_slice(_device_tensor(g, "mm_gt"), t0, t, 1).reshape(g.shape[0], T, -1) for g in mm_gt if g.shape[0]]
    for g in parts:
        if g.shape[2] != F:
            raise ValueError(f"mm_gt frames have {g.shape[2]} features, pred frames {F}")
    gts = torch.cat(parts).contiguous() if parts else torch.empty((0, T, F), device=dev)
    npairs = gts.shape[0]
    cnt = torch.tensor(counts, dtype=torch.int64)
    off = torch.zeros(B + 1, dtype=torch.int64)
    off[1:] = torch.cumsum(cnt, 0)
    off = off.to(dev)
    pair_seq = torch.repeat_interleave(torch.arange(B, dtype=torch.int64), cnt).to(dev)
    pair = torch.empty(max(npairs, 1), device=dev, dtype=torch.float32)
    out = torch.empty(B, device=dev, dtype=torch.float32)
    stream = torch.cuda.current_stream(dev).cuda_stream
    args = (pair, None, out, None) if want_ade else (None, pair, None, out)
    check(_lib.lib().sd_mm_ade_fde(p.data_ptr(), gts.data_ptr() if npairs else None, pair_seq.data_ptr() if npairs else None,
                                   npairs, off.data_ptr(), B, S, T, F, *(_lib.ptr(a) for a in args), stream))
    return out


def mmade(target: torch.Tensor, pred: torch.Tensor, mm_gt, t0: int = 0, t: int = -1, **kwargs) -> torch.Tensor:
    """Multimodal ADE (multimodal.py:108-120): pred (batch, num_samples, seq_length, ...), mm_gt a
    sequence of batch tensors (n_gts_i, seq_length, ...): per sequence the mean over its ground
    truths of the min over samples of the mean-over-frames L2 distance (RuntimeError for a
    sequence without ground truths, as the reference).  `target` is unused, as in the reference."""
    return _mm(target, pred, mm_gt, t0, t, True)


def mmfde(target: torch.Tensor, pred: torch.Tensor, mm_gt, t0: int = 0, t: int = -1, **kwargs) -> torch.Tensor:
    """Multimodal FDE (multimodal.py:122-135): as mmade on the last frame of the slice."""
    return _mm(target, pred, mm_gt, t0, t, False)


__all__ = ["lat_apd", "apd", "ade", "fde", "mmade", "mmfde"]
