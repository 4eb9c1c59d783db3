"""Checkpoint I/O at the sampler's boundary (SURVEY.md §8f "next" #3).

The reference's training run saves ``{'model': diffusion.state_dict(), 'opt': ..., 'trainer': ...}``
through ignite's ``Checkpoint`` as ``checkpoints/checkpoint_<epoch>[_val_ade=...].pt``
(``train_diffusion.py:100-103``, ``src/core/trainer.py:168-176``), finds the newest ``checkpoint_<epoch>*.pt`` of a run
(``src/utils/load.py:4-9``) and loads it strictly into the freshly built diffusion
(``eval_prepare_model.py:69-72``).  The same keys (the 18 diffusion buffers + ``model.*``, 137 for
the release Denoiser) load here, and the sampling plan is rebuilt from them on the next call.

Difference by design: files are read with ``torch.load(..., weights_only=True)`` -- tensors and
plain containers only, nothing in the file is executed.  A checkpoint that needs arbitrary
unpickling (the reference's plain ``torch.load``) is refused with the loader's own error.
"""
from __future__ import annotations

import os
from typing import Any, Dict, Optional

import torch

__all__ = ["get_latest_model_path", "load_model_checkpoint", "load_diffusion_checkpoint",
           "save_diffusion_checkpoint"]


def get_latest_model_path(ckpnt_path: str) -> str:
    """Path of the highest-epoch ``checkpoint_<epoch>[...].pt`` in a run directory
    (``src/utils/load.py:4-9``: the epoch is the text between ``checkpoint_`` and ``_val`` /
    ``.pt``)."""
    files = [f for f in os.listdir(ckpnt_path) if f.startswith("checkpoint_")]
    if not files:
        raise FileNotFoundError(f"no checkpoint_* file in {ckpnt_path}")
    epoch = {int(f.split("_val")[0].replace("checkpoint_", "").replace(".pt", "")): f for f in files}
    return os.path.join(ckpnt_path, epoch[max(epoch)])


def load_model_checkpoint(load_path: str, map_location: Any = "cpu") -> Dict[str, Any]:
    """The checkpoint dict (``src/utils/load.py:11-17``), read with the tensor-only loader."""
    return torch.load(load_path, map_location=map_location, weights_only=True)


def load_diffusion_checkpoint(diffusion: torch.nn.Module, load_path: str, strict: bool = True,
                              map_location: Any = "cpu") -> Dict[str, Any]:
    """``diffusion.load_state_dict(checkpoint['model'])`` (``eval_prepare_model.py:69-72``).
    Accepts a bare state_dict as well.  Returns the checkpoint dict (other entries: epoch,
    optimizer state, ... as the training run saved them)."""
    ckpt = load_model_checkpoint(load_path, map_location=map_location)
    sd = ckpt["model"] if isinstance(ckpt, dict) and "model" in ckpt else ckpt
    diffusion.load_state_dict(sd, strict=strict)
    return ckpt


def save_diffusion_checkpoint(diffusion: torch.nn.Module, path: str, epoch: Optional[int] = None,
                              **extra: Any) -> None:
    """Write ``{'model': state_dict, 'epoch': epoch, **extra}`` (the ``'model'`` entry of the
    reference's checkpoint objects, ``src/core/trainer.py:168-176``), tensors moved to the CPU."""
    sd = {k: v.detach().cpu() for k, v in diffusion.state_dict().items()}
    obj: Dict[str, Any] = {"model": sd}
    if epoch is not None:
        obj["epoch"] = int(epoch)
    obj.update(extra)
    torch.save(obj, path)
