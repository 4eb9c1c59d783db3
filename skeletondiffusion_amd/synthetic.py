"""Deterministic synthetic weights and inputs for benchmarks and parity fixtures.

No checkpoint can be fetched in this environment (`README.md:156` of the
reference points at a remote HF repo), so every benchmark and every golden fixture runs on
weights produced by this filler.  It is pure numpy (PCG64), so the same seed gives the same
bytes on the build container and on the GPU box; only the outputs of the reference are
committed as fixtures, never the weights.

Filling rule (one PCG64 stream, parameters visited in sorted-name order):
  * ``*.G``   (learnable graph influence, `graph_structural.py:333-334`): I + U(0, 0.1)
  * ``*.g``   (RMSNorm gain, `attention.py:30-36`):                       1 + U(-0.1, 0.1)
  * ``*weight``: U(-1/sqrt(fan_in), 1/sqrt(fan_in)), fan_in = last dim (in_features)
  * ``*bias`` : U(-0.1, 0.1)
Buffers (e.g. the identity ``G`` of a non-learnable StaticGraphLinear) are not touched.
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, Tuple

import numpy as np


def fill_parameters(named_shapes: Iterable[Tuple[str, Tuple[int, ...]]], seed: int) -> Dict[str, np.ndarray]:
    """Return {name: float32 array} for every (name, shape) given (parameters only)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out: Dict[str, np.ndarray] = {}
    for name, shape in sorted(named_shapes, key=lambda kv: kv[0]):
        shape = tuple(int(s) for s in shape)
        leaf = name.rsplit(".", 1)[-1]
        if leaf == "G":
            a = np.eye(shape[0], shape[1]) + rng.uniform(0.0, 0.1, size=shape)
        elif leaf == "g":
            a = 1.0 + rng.uniform(-0.1, 0.1, size=shape)
        elif leaf == "G_add":  # additive graph influence of the GRU cells (recurrent.py:236-245)
            a = rng.uniform(-0.05, 0.05, size=shape)
        elif leaf in ("weight", "weight_ih", "weight_hh"):
            bound = 1.0 / math.sqrt(shape[-1])
            a = rng.uniform(-bound, bound, size=shape)
        elif leaf in ("bias", "bias_ih", "bias_hh"):
            a = rng.uniform(-0.1, 0.1, size=shape)
        else:
            raise KeyError(f"synthetic filler has no rule for parameter {name!r}")
        out[name] = a.astype(np.float32)
    return out


def fill_module_(module, seed: int) -> None:
    """Overwrite every parameter of a torch module in place with the synthetic filler."""
    import torch

    named = [(n, tuple(p.shape)) for n, p in module.named_parameters()]
    vals = fill_parameters(named, seed)
    with torch.no_grad():
        for n, p in module.named_parameters():
            p.copy_(torch.from_numpy(vals[n]))


def normal(shape, seed: int) -> np.ndarray:
    """Standard-normal float32 array from PCG64 (used for start/sampling noise fixtures)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.standard_normal(size=tuple(shape)).astype(np.float32)


def uniform(shape, seed: int, low: float = -1.0, high: float = 1.0) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    return rng.uniform(low, high, size=tuple(shape)).astype(np.float32)


def readme_correlation(num_nodes: int, seed: int) -> np.ndarray:
    """The README plug-and-play correlation recipe (`README.md:83-84`), drawn from PCG64:
    rand >= 0.5 -> binary A; corr = (A + A.T) // 2 (symmetric)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    a = (rng.random((num_nodes, num_nodes)) >= 0.5).astype(np.float32)
    return np.floor_divide(a + a.T, 2).astype(np.float32)
