"""NonisotropicGaussianDiffusion with the reference API and state_dict
(reference src/core/diffusion/nonisotropic.py:5-227).

Everything here is host-side setup (the 14 Sigma-derived buffers, computed once, in the
reference's op order so the buffers are bit-identical) plus the torch-op training helpers.
The per-step posterior update that sampling needs is the HIP kernel `k_update`
(C1[t] x0 + C2[t] x_t + U (sigma_t . eps)), reached through the engine.
"""
from __future__ import annotations

import torch

from ... import training as _training
from .base import LatentDiffusion, default, extract

__all__ = ["NonisotropicGaussianDiffusion", "compute_covariance_matrices", "extract_matrix"]


def extract_matrix(matrix, t, x_shape):
    """matrix[t] as a (B, ...) batch broadcastable against x_shape (nonisotropic.py:5-12)."""
    out = torch.index_select(matrix, 0, t)
    while len(x_shape) > out.dim():
        out = out.unsqueeze(-1)
    return out


def _rows_times(d, M):  # diag(d) @ M for a batch of diagonals d (T, N)
    return d.unsqueeze(-1) * M


def _cols_times(M, d):  # M @ diag(d)
    return M * d.unsqueeze(-2)


def compute_covariance_matrices(diffusion, Lambda_N, diffusion_covariance_type="skeleton-diffusion",
                                gamma_scheduler="cosine"):
    """(Lambda_t, Lambda_bar_t, Lambda_bar_{t-1}), each (T, N)  (nonisotropic.py:36-68).
    Uses the fp32 registered schedule buffers, exactly as the reference does."""
    N = Lambda_N.shape[0]
    alphas = 1.0 - diffusion.betas
    ac = diffusion.alphas_cumprod
    T = alphas.shape[0]
    diffusion.alphas_sumprod = torch.stack(
        [torch.sum(torch.cumprod(torch.flip(alphas[: t + 1], [0]), dim=0)) for t in range(T)], dim=0)
    if diffusion_covariance_type == "isotropic":
        assert (Lambda_N == 0).all()
        lam_t = (1 - alphas).unsqueeze(-1)
        lam_bar = 1 - ac.unsqueeze(-1)
        lam_prev = torch.cat([torch.zeros(1).unsqueeze(0), lam_bar[:-1]], dim=0)
        return lam_t, lam_bar, lam_prev
    if diffusion_covariance_type == "anisotropic":
        return ((1 - alphas.unsqueeze(-1)) * Lambda_N, (1 - ac.unsqueeze(-1)) * Lambda_N,
                (1 - diffusion.alphas_cumprod_prev.unsqueeze(-1)) * Lambda_N)
    if diffusion_covariance_type != "skeleton-diffusion":
        raise AssertionError("Not implemented")
    if gamma_scheduler == "cosine":
        gammas = 1 - alphas
    elif gamma_scheduler == "mono_decrease":
        gammas = 1 - torch.arange(0, diffusion.num_timesteps) / diffusion.num_timesteps
    else:
        raise AssertionError("Not implemented")
    lam_i = Lambda_N - 1
    g_bar = (1 - alphas) * gammas
    g_tilde = ac * torch.cumsum(g_bar / ac, dim=-1)
    lam_t = lam_i.unsqueeze(0) * g_bar.unsqueeze(-1) + (1 - alphas).unsqueeze(-1)
    lam_bar = lam_i.unsqueeze(0) * g_tilde.unsqueeze(-1) + (1 - ac.unsqueeze(-1))
    lam_prev = torch.cat([torch.zeros(N).unsqueeze(0), lam_bar[:-1]], dim=0)  # deterministic start
    return lam_t, lam_bar, lam_prev


class NonisotropicGaussianDiffusion(LatentDiffusion):
    def __init__(self, Sigma_N: torch.Tensor, Lambda_N: torch.Tensor, U: torch.Tensor,
                 diffusion_covariance_type="skeleton-diffusion", loss_reduction_type="l1",
                 gamma_scheduler="cosine", **kwargs):
        super().__init__(**kwargs)
        self.diffusion_covariance_type = diffusion_covariance_type
        self._register("Lambda_N", Lambda_N)
        self._register("Sigma_N", Sigma_N)
        self.set_rotation_matrix(U)
        lam_t, lam_bar, lam_prev = compute_covariance_matrices(self, Lambda_N, diffusion_covariance_type,
                                                               gamma_scheduler)
        Ut = self.U_transposed.unsqueeze(0)
        U0 = U.unsqueeze(0)
        alphas = 1.0 - self.betas

        def diag_stack(v):
            return torch.stack([torch.diag(d) for d in v], dim=0)

        # noise <-> x0 conversions (predict_noise_from_start / predict_start_from_noise)
        self._register("inv_sqrt_Lambda_bar_mmUt", _rows_times(1 / torch.sqrt(lam_bar), Ut))
        self._register("inv_sqrt_Lambda_bar_sqrt_alphas_cumprod_mmUt",
                       _rows_times((1 / torch.sqrt(lam_bar)) * self.sqrt_alphas_cumprod.unsqueeze(-1), Ut))
        self._register("Umm_sqrt_Lambda_bar_t", _cols_times(U0, torch.sqrt(lam_bar)))
        self._register("Umm_sqrt_Lambda_bar_t_sqrt_recip_alphas_cumprod",
                       _cols_times(U0, torch.sqrt(lam_bar / self.alphas_cumprod.unsqueeze(-1))))
        # posterior q(x_{t-1} | x_t, x0)
        lam_post = lam_t * lam_prev * (1 / lam_bar)
        self._register("Lambda_posterior", lam_post)
        self._register("Lambda_posterior_log_variance_clipped", torch.log(lam_post.clamp(min=1e-20)))
        c1 = torch.sqrt(self.alphas_cumprod_prev).unsqueeze(-1).unsqueeze(-1) * \
            (U0 @ diag_stack((1 / lam_bar) * lam_t) @ Ut)
        c2 = torch.sqrt(alphas).unsqueeze(-1).unsqueeze(-1) * (U0 @ diag_stack((1 / lam_bar) * lam_prev) @ Ut)
        self._register("posterior_mean_coef1_x0", c1)
        self._register("posterior_mean_coef2_xt", c2)
        # Mahalanobis loss
        self.loss_reduction_type = loss_reduction_type
        self._register("mahalanobis_S_sqrt_recip", _rows_times(torch.sqrt(1.0 / lam_bar), Ut))
        if self.objective == "pred_noise":
            loss_weight = torch.ones_like(alphas)
        elif self.objective == "pred_x0":
            loss_weight = self.alphas_cumprod
        else:
            raise AssertionError("Not implemented")  # pred_v (nonisotropic.py:122-123)
        self._register("loss_weight", loss_weight)
        assert self.mahalanobis_S_sqrt_recip.dim() != 1

    def set_rotation_matrix(self, U: torch.Tensor):
        self._register("U", U)
        self._register("U_transposed", U.t())

    def check_eigh(self):
        return torch.isclose(self.U @ torch.diag(self.Lambda_N) @ self.U_transposed, self.Sigma_N)

    def get_anisotropic_noise(self, x, *args, **kwargs):
        return self.get_noise(x, *args, **kwargs) * self.Lambda_N.unsqueeze(-1)

    # -- forward process ----------------------------------------------------------------------
    def q_sample(self, x_start, t, noise=None):
        noise = default(noise, lambda: self.get_white_noise(x_start))
        return (extract(self.sqrt_alphas_cumprod, t, x_start.shape) * x_start +
                extract_matrix(self.Umm_sqrt_Lambda_bar_t, t, x_start.shape) @ noise)

    def predict_start_from_noise(self, x_t, t, noise):
        # the reference reads self.sqrt_recip_alphas_cumprod, which this class never registers
        # (nonisotropic.py:161-165): pred_noise is unusable there; kept failing the same way.
        raise AttributeError("'NonisotropicGaussianDiffusion' has no buffer 'sqrt_recip_alphas_cumprod' "
                             "(reference nonisotropic.py:163)")

    def predict_noise_from_start(self, x_t, t, x0):
        return (extract_matrix(self.inv_sqrt_Lambda_bar_mmUt, t, x_t.shape) @ x_t -
                extract_matrix(self.inv_sqrt_Lambda_bar_sqrt_alphas_cumprod_mmUt, t, x_t.shape) @ x0)

    # -- loss ---------------------------------------------------------------------------------
    def mahalanobis_dist(self, matrix, vector):
        return (matrix @ vector).abs()

    def loss_funct(self, model_out, target, t):
        diff = target - model_out if self.objective == "pred_noise" else model_out - target
        loss = self.mahalanobis_dist(extract_matrix(self.mahalanobis_S_sqrt_recip, t, diff.shape), diff)
        if self.loss_reduction_type == "l1":
            return loss
        if self.loss_reduction_type == "mse":
            return loss ** 2
        raise AssertionError("Not implemented")

    def loss_rows(self, model_out, target, t):
        """The Mahalanobis loss reduced per row.  On the device under autograd (fp32, J <= 64,
        F <= 256, loss_funct not overridden) it is one fused HIP kernel each way
        (training.mahalanobis_loss, sd_train.hip `k_mahalanobis`); otherwise loss_funct + mean."""
        if (model_out.is_cuda and torch.is_grad_enabled() and model_out.dtype == torch.float32 and model_out.dim() == 3
                and _training.hip_training_enabled() and type(self).loss_funct is NonisotropicGaussianDiffusion.loss_funct
                and self.loss_reduction_type in ("l1", "mse") and self.objective in ("pred_noise", "pred_x0")
                and model_out.shape[1] <= _training.MAX_NODES and model_out.shape[2] <= 256
                and self.mahalanobis_S_sqrt_recip.dtype == torch.float32 and target.shape == model_out.shape
                and t.numel() == model_out.shape[0]):
            return _training.mahalanobis_loss(model_out, target, self.mahalanobis_S_sqrt_recip, t.reshape(-1),
                                              self.objective == "pred_noise", self.loss_reduction_type == "mse")
        return super().loss_rows(model_out, target, t)

    # -- reverse process (torch reference forms of the HIP update) -------------------------------
    def q_posterior_mean(self, x_start, x_t, t):
        return (extract_matrix(self.posterior_mean_coef1_x0, t, x_t.shape) @ x_start +
                extract_matrix(self.posterior_mean_coef2_xt, t, x_t.shape) @ x_t)

    def q_posterior(self, x_start, x_t, t):
        return (self.q_posterior_mean(x_start, x_t, t),
                extract_matrix(self.Lambda_posterior, t, x_t.shape),
                extract_matrix(self.Lambda_posterior_log_variance_clipped, t, x_t.shape))

    def p_combine_mean_var_noise(self, model_mean, posterior_log_variance, noise):
        """mean (joint coordinates) + U (sigma . eps) (sigma in the eigenbasis)."""
        return model_mean + self.U @ ((0.5 * posterior_log_variance).exp() * noise)

    def interpolate_noise(self, noise1, noise2, posterior_log_variance=None, interpolate_funct=None):
        s = (0.5 * posterior_log_variance).exp()
        return interpolate_funct(self.U @ (s * noise1), self.U @ (s * noise2))

    def p_interpolate_mean_var_noise(self, model_mean, model_log_variance, noise, noise2interpolate=None, **kwargs):
        return model_mean + self.interpolate_noise(noise, noise2interpolate,
                                                   posterior_log_variance=model_log_variance, **kwargs)
