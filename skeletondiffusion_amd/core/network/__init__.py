"""Mirror of `src.core.network` (reference src/core/network/nn/__init__.py): the Denoiser."""
from .layers import (Attention, PreNorm, Residual, ResnetBlock, RMSNorm, StaticGraphLinear,
                     SinusoidalPosEmb)
from .generator import Denoiser

__all__ = ["Denoiser", "StaticGraphLinear", "Attention", "ResnetBlock", "Residual", "PreNorm",
           "RMSNorm", "SinusoidalPosEmb"]
