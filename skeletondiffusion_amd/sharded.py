"""Batched multi-future evaluation sharded over the GPUs of a node.

One process per GPU (``torchrun``; ``torch.distributed`` backend ``"nccl"`` = RCCL over xGMI).
Rows never interact, so the only collectives are at the edges of the sampling:

* ``broadcast_state``: rank 0's diffusion state_dict (weights + Σ/Λ/U buffers) to every rank,
  once, so all shards sample with identical parameters (one broadcast per tensor, bucketed into
  one flat buffer per dtype);
* ``sample_sharded``: rank r samples sequences ``shard_range(nseq, r, world)`` with all their
  futures (``eval_prepare_model.py:96`` repeat_interleave order) and ``row0`` = its first global
  row, so the device Philox noise -- and the latents -- do not depend on the GPU count; the
  shards are then gathered (``all_gather`` of padded shards: ragged when ``nseq`` does not
  divide by the world size) or kept local;
* ``reduce_metric``: per-sequence metric values (e.g. ``metrics.apd``) summed over ranks with one
  ``all_reduce`` -> the dataset mean without moving the latents.

The reference evaluates with one process and ``DataParallel`` (broken for ``.sample``,
SURVEY.md §2.2); this replaces that with sequence sharding.
"""
from __future__ import annotations

from typing import Callable, Dict, Optional, Tuple

import torch
import torch.distributed as dist

__all__ = ["shard_range", "broadcast_state", "sample_sharded", "reduce_metric"]


def shard_range(nseq: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous, balanced sequence shard [s0, s1) of `rank`: the first nseq % world ranks take
    one sequence more (11,015 sequences over 8 GPUs -> 1,377 x 7 + 1,376)."""
    if not (0 <= rank < world):
        raise ValueError(f"rank {rank} outside world {world}")
    base, extra = divmod(nseq, world)
    s0 = rank * base + min(rank, extra)
    return s0, s0 + base + (1 if rank < extra else 0)


def _world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def broadcast_state(module: torch.nn.Module, src: int = 0) -> None:
    """Every rank's `module` takes `src`'s parameters and buffers (in place), one flat broadcast
    per dtype.  No-op without an initialised process group."""
    rank, world = _world()
    if world == 1:
        return
    tensors = [t for t in module.state_dict(keep_vars=True).values() if torch.is_tensor(t)]
    by_dtype: Dict[torch.dtype, list] = {}
    for t in tensors:
        by_dtype.setdefault(t.dtype, []).append(t)
    with torch.no_grad():
        for dtype, ts in by_dtype.items():
            flat = torch.cat([t.detach().reshape(-1) for t in ts])
            dist.broadcast(flat, src)
            off = 0
            for t in ts:
                n = t.numel()
                t.data.copy_(flat[off:off + n].view_as(t))
                off += n


def sample_sharded(sample_fn: Callable[..., torch.Tensor], x_cond: torch.Tensor, futures: int,
                   seed: int, gather: bool = True) -> Tuple[torch.Tensor, int]:
    """Sample this rank's shard of `x_cond` (all sequences, (nseq, J, D), on this rank's device)
    with `futures` futures per sequence.  `sample_fn(batch_size=, x_cond=, seed=, row0=)` returns
    (rows, J, D) latents -- normally ``lambda **kw: diffusion.sample(**kw)[0]``.
    Returns (latents, s0): all nseq*futures rows in sequence order on every rank when `gather`,
    else this rank's rows and its first sequence s0."""
    rank, world = _world()
    nseq = x_cond.shape[0]
    s0, s1 = shard_range(nseq, rank, world)
    if s1 > s0:
        mine = sample_fn(batch_size=(s1 - s0) * futures, x_cond=x_cond[s0:s1], seed=seed, row0=s0 * futures)
    else:  # more ranks than sequences: an empty shard still joins the all_gather below
        mine = x_cond.new_empty((0,) + tuple(x_cond.shape[1:]))
    if not gather or world == 1:
        return mine, s0
    # ragged shards: pad to the largest shard, all_gather, then drop the padding
    per = [shard_range(nseq, r, world) for r in range(world)]
    rows_max = max(b - a for a, b in per) * futures
    if rows_max == 0:
        return mine, s0
    buf = mine.new_zeros((rows_max,) + tuple(mine.shape[1:]))
    buf[:mine.shape[0]] = mine
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    out = torch.cat([p[:(b - a) * futures] for p, (a, b) in zip(parts, per)])
    return out, s0


def reduce_metric(values: torch.Tensor, nseq_total: Optional[int] = None) -> torch.Tensor:
    """Mean over all sequences of per-sequence metric `values` (this rank's shard, (n_local,)):
    one all_reduce of [sum, count] in float64."""
    acc = torch.stack([values.double().sum(), torch.tensor(float(values.numel()), dtype=torch.float64,
                                                           device=values.device)])
    rank, world = _world()
    if world > 1:
        dist.all_reduce(acc)
    if nseq_total is not None and int(acc[1].item()) != nseq_total:
        raise RuntimeError(f"reduced {int(acc[1].item())} sequences, expected {nseq_total}")
    return (acc[0] / acc[1]).float()
