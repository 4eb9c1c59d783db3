"""MI355X-native nonisotropic latent-diffusion sampler (SkeletonDiffusion hot path)."""
__version__ = "0.1.0"
