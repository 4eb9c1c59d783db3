"""Mirror of `src.core.diffusion` (reference src/core/diffusion/__init__.py:1-3)."""
from .isotropic import IsotropicGaussianDiffusion
from .nonisotropic import NonisotropicGaussianDiffusion
from .utils import get_cov_from_corr

__all__ = ["IsotropicGaussianDiffusion", "NonisotropicGaussianDiffusion", "get_cov_from_corr"]
