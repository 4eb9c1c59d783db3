"""LatentDiffusion: schedules, the training forward, and the reverse loop, with the reference
API (src/core/diffusion/base.py:64-443).

Sampling (`sample`, `p_sample_loop`, `p_sample`, `p_mean_variance`) runs on the MI355X HIP
engine (skeletondiffusion_amd/engine.py -> libskeldiff.so).  There is no CPU sampling path:
calling them with the module on the CPU raises.  The training path (`forward` / `p_losses`)
stays on torch ops so that it keeps autograd.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch
import torch.nn.functional as F
from torch import nn

from ... import engine as _engine

__all__ = ["LatentDiffusion", "extract", "default", "exists", "identity", "linear_beta_schedule",
           "cosine_beta_schedule", "exp_beta_schedule", "ModelPrediction"]

from collections import namedtuple

ModelPrediction = namedtuple("ModelPrediction", ["pred_noise", "pred_x_start"])


def identity(t, *args, **kwargs):
    return t


def exists(x):
    return x is not None


def default(val, d):
    if exists(val):
        return val
    return d() if callable(d) else d


def extract(a, t, x_shape):
    """a[t] reshaped to broadcast against x_shape (base.py:34-37)."""
    out = a.gather(-1, t)
    return out.reshape(t.shape[0], *((1,) * (len(x_shape) - 1)))


def linear_beta_schedule(timesteps):
    scale = 1000 / timesteps
    return torch.linspace(scale * 0.0001, scale * 0.02, timesteps, dtype=torch.float64)


def cosine_beta_schedule(timesteps, s=0.008):
    """Nichol & Dhariwal cosine schedule, clipped to 0.999 (base.py:45-55)."""
    x = torch.linspace(0, timesteps, timesteps + 1, dtype=torch.float64)
    ac = torch.cos(((x / timesteps) + s) / (1 + s) * math.pi * 0.5) ** 2
    ac = ac / ac[0]
    return torch.clip(1 - (ac[1:] / ac[:-1]), 0, 0.999)


def exp_beta_schedule(timesteps, factor=3.0):
    x = torch.linspace(-factor, 0, timesteps + 1, dtype=torch.float64)
    return torch.clip(torch.exp(x), 0, 0.999)


_SCHEDULES = {"linear": lambda T, f: linear_beta_schedule(T),
              "cosine": lambda T, f: cosine_beta_schedule(T),
              "exp": lambda T, f: exp_beta_schedule(T, f)}


class LatentDiffusion(nn.Module):
    def __init__(self, model: nn.Module, latent_size=96, diffusion_timesteps=10, diffusion_objective="pred_x0",
                 sampling_timesteps=None, diffusion_activation="identity", diffusion_conditioning=False,
                 diffusion_loss_type="mse", objective="pred_noise", beta_schedule="cosine",
                 beta_schedule_factor=3.0, ddim_sampling_eta=0.0, **kwargs):
        super().__init__()
        if diffusion_activation == "tanh":
            self.activation = nn.Tanh()
        elif diffusion_activation == "identity":
            self.activation = nn.Identity()
        self.diffusion_activation = diffusion_activation
        self.silent = True
        self.condition = diffusion_conditioning
        self.loss_type = diffusion_loss_type
        self.statistics_pred = None
        self.statistics_obs = None

        self.model = model
        self.channels = model.channels
        self.self_condition = model.self_condition
        self.seq_length = latent_size
        self.objective = diffusion_objective  # the `objective` kwarg is overridden (base.py:90-91)
        assert self.objective in {"pred_noise", "pred_x0", "pred_v"}, \
            "objective must be either pred_noise, pred_x0 or pred_v"
        if beta_schedule not in _SCHEDULES:
            raise ValueError(f"unknown beta schedule {beta_schedule}")
        betas = _SCHEDULES[beta_schedule](diffusion_timesteps, beta_schedule_factor)
        alphas = 1.0 - betas
        ac = torch.cumprod(alphas, dim=0)
        ac_prev = F.pad(ac[:-1], (1, 0), value=1.0)
        self.num_timesteps = int(betas.shape[0])
        self.sampling_timesteps = default(sampling_timesteps, self.num_timesteps)
        assert self.sampling_timesteps <= self.num_timesteps
        self.is_ddim_sampling = self.sampling_timesteps < self.num_timesteps
        self.ddim_sampling_eta = ddim_sampling_eta
        self._register("betas", betas)
        self._register("alphas_cumprod", ac)
        self._register("alphas_cumprod_prev", ac_prev)
        self._register("sqrt_alphas_cumprod", torch.sqrt(ac))
        self._engine = None

    # -- helpers --------------------------------------------------------------------------
    def _register(self, name, value):
        self.register_buffer(name, value.to(torch.float32))

    def set_normalization_statistics(self, statistics_pred, statistics_obs):
        self.statistics_pred = statistics_pred
        self.statistics_obs = statistics_obs

    def get_noise(self, x, *args, **kwargs):
        if torch.is_tensor(x):
            return torch.randn_like(x)
        if isinstance(x, tuple):
            return torch.randn(*x, *args, **kwargs)

    def get_white_noise(self, x, *args, **kwargs):
        return self.get_noise(x, *args, **kwargs)

    def get_start_noise(self, x, *args, **kwargs):
        return self.get_white_noise(x, *args, **kwargs)

    # -- subclass interface -----------------------------------------------------------------
    def predict_start_from_noise(self, x_t, t, noise):
        raise AssertionError("Not implemented")

    def predict_noise_from_start(self, x_t, t, x0):
        raise AssertionError("Not implemented")

    def predict_v(self, x_start, t, noise):
        raise AssertionError("Not implemented")

    def predict_start_from_v(self, x_t, t, v):
        raise AssertionError("Not implemented")

    def q_sample(self, x_start, t, noise=None):
        raise AssertionError("Not implemented")

    def q_posterior(self, x_start, x_t, t):
        raise AssertionError("Not implemented")

    def p_combine_mean_var_noise(self, model_mean, model_log_variance, noise):
        raise AssertionError("Not implemented")

    def p_interpolate_mean_var_noise(self, model_mean, model_log_variance, noise, noise2interpolate=None, **kwargs):
        raise AssertionError("Not implemented")

    def loss_funct(self, model_out, target, *args, **kwargs):
        if self.loss_type == "mse":
            return F.mse_loss(model_out, target, reduction="none")
        if self.loss_type == "l1":
            return F.l1_loss(model_out, target, reduction="none")
        raise AssertionError("Not implemented")

    # -- network interface (torch / autograd) ------------------------------------------------
    def feed_model(self, x, t, x_self_cond=None, x_cond=None):
        if self.condition:
            assert x_cond is not None
            if x.shape[0] > x_cond.shape[0]:
                x_cond = x_cond.repeat_interleave(int(x.shape[0] / x_cond.shape[0]), 0)
        return self.activation(self.model(x, t, x_self_cond, x_cond))

    def model_predictions(self, x, t, x_self_cond=None, x_cond=None, clip_x_start=False, rederive_pred_noise=False):
        out = self.feed_model(x, t, x_self_cond=x_self_cond, x_cond=x_cond)
        clip = (lambda v: torch.clamp(v, -1.0, 1.0)) if clip_x_start else identity
        if self.objective == "pred_noise":
            pred_noise = out
            x_start = clip(self.predict_start_from_noise(x, t, pred_noise))
            if clip_x_start and rederive_pred_noise:
                pred_noise = self.predict_noise_from_start(x, t, x_start)
        elif self.objective == "pred_x0":
            x_start = clip(out)
            pred_noise = self.predict_noise_from_start(x, t, x_start)
        else:
            x_start = clip(self.predict_start_from_v(x, t, out))
            pred_noise = self.predict_noise_from_start(x, t, x_start)
        return ModelPrediction(pred_noise, x_start)

    # -- forward process (training) -----------------------------------------------------------
    def loss_rows(self, model_out, target, t):
        """loss_funct reduced 'b ... -> b' by the mean (reference base.py:297-298)."""
        loss = self.loss_funct(model_out, target, t)
        return loss.reshape(loss.shape[0], -1).mean(dim=1)

    def p_losses(self, x_start, t, noise=None, x_cond=None, n_train_samples=1):
        b = x_start.shape[0]
        if n_train_samples > 1:
            x_start = x_start.repeat_interleave(n_train_samples, dim=0)
            t = t.repeat_interleave(n_train_samples, dim=0)
            if x_cond is not None:
                x_cond = x_cond.repeat_interleave(n_train_samples, dim=0)
        noise = default(noise, lambda: self.get_white_noise(x_start, t))
        x = self.q_sample(x_start=x_start, t=t, noise=noise)
        x_self_cond = None
        if self.self_condition and torch.rand(()) < 0.5:
            with torch.no_grad():
                x_self_cond = self.model_predictions(x, t, x_cond=x_cond).pred_x_start.detach()
        model_out = self.feed_model(x, t, x_self_cond=x_self_cond, x_cond=x_cond)
        if self.objective == "pred_noise":
            target = noise
        elif self.objective == "pred_x0":
            target = x_start
        elif self.objective == "pred_v":
            target = self.predict_v(x_start, t, noise)
        else:
            raise ValueError(f"unknown objective {self.objective}")
        loss = self.loss_rows(model_out, target, t)
        return loss, extract(self.loss_weight, t.view(b, -1)[:, 0], loss.shape[0:1]), model_out

    def forward(self, x, *args, x_cond=None, **kwargs):
        b, c, n = x.shape
        assert n == self.seq_length, f"seq length must be {self.seq_length}"
        t = torch.randint(0, self.num_timesteps, (b,), device=x.device).long()
        return self.p_losses(x, t, *args, x_cond=x_cond, **kwargs)

    # -- reverse process (HIP engine) ---------------------------------------------------------
    @property
    def engine(self) -> "_engine.SamplingEngine":
        if self._engine is None:
            self._engine = _engine.SamplingEngine(self)
        return self._engine

    @torch.no_grad()
    def p_mean_variance(self, x, t, x_self_cond=None, x_cond=None, clip_denoised=True):
        """base.py:314-322: x0 from the Denoiser output (HIP engine) per objective, as
        model_predictions forms it (base.py:219-241: the activation, then predict_start_from_noise /
        predict_start_from_v for pred_noise / pred_v), clamped unless clip_denoised=False, then the
        posterior q(x_{t-1} | x_t, x0)."""
        tt = int(t[0]) if torch.is_tensor(t) else int(t)
        out = self.engine.denoiser_forward(x, tt, x_cond)
        x_start = self.engine.start_from_output(x, tt, out)
        if clip_denoised:
            x_start.clamp_(-1.0, 1.0)
        t_b = torch.full((x.shape[0],), tt, device=x.device, dtype=torch.long)
        mean, var, logvar = self.q_posterior(x_start=x_start, x_t=x, t=t_b)
        return mean, var, logvar, x_start

    @torch.no_grad()
    def p_sample(self, x, t: int, x_self_cond=None, clip_denoised=True, sampling_noise=None, *args,
                 if_interpolate=False, noise2interpolate=None, interpolation_kwargs: Dict = None, x_cond=None,
                 **kwargs):
        """One reverse step (base.py:324-341): returns (x_{t-1}, x0, noise, mean)."""
        if if_interpolate and t > 0:
            mean, _, logvar, x_start = self.p_mean_variance(x, t, x_self_cond, x_cond=x_cond,
                                                            clip_denoised=clip_denoised)
            noise = sampling_noise[:, sampling_noise.shape[1] - t] if sampling_noise is not None \
                else self.get_white_noise(x)
            noise2 = noise2interpolate[:, noise2interpolate.shape[1] - t]
            assert noise2.shape == noise.shape
            img = self.p_interpolate_mean_var_noise(mean, logvar, noise, noise2, **(interpolation_kwargs or {}))
            return img, x_start, noise, mean
        eps = None
        if t > 0:
            eps = sampling_noise[:, sampling_noise.shape[1] - t] if sampling_noise is not None \
                else self.get_white_noise(x)
        return self.engine.p_sample(x, t, x_cond, eps, clip=bool(clip_denoised))

    @torch.no_grad()
    def p_sample_loop(self, shape, x_cond=None, start_noise=None, sampling_noise=None,
                      return_sampling_noise=False, return_timages=False, if_interpolate=False,
                      noise2interpolate=None, interpolation_kwargs=None, seed=None, row0=0, out=None, **kwargs):
        """Reverse chain t = T-1 .. 0 (base.py:343-390) on the HIP engine.

        Engine extensions (keyword-only, optional): `seed` fixes the device Philox stream used
        when start/sampling noise is not supplied (default: drawn from torch's global RNG, so
        torch.manual_seed controls it); `row0` is the global index of the first row, which makes
        device noise independent of how rows are split over launches or GPUs; `out` (rows, J, D)
        fp32 receives the latents (reusing it keeps a captured hipGraph valid across calls).
        `clip_denoised` (default True) travels in **kwargs to p_sample, as in the reference
        (base.py:344,367 -> :325); False leaves x0 unclamped (SD_FLAG_NO_CLIP)."""
        clip = bool(kwargs.pop("clip_denoised", True))
        if start_noise is not None:
            assert tuple(start_noise.shape) == tuple(shape), f"Shape mismatch: {start_noise.shape} != {shape}"
        if sampling_noise is not None:
            assert sampling_noise.shape[2:] == shape[1:], f"Shape mismatch: {sampling_noise.shape} != {shape}"
            assert sampling_noise.shape[0] == shape[0], f"Shape mismatch: {sampling_noise.shape} != {shape}"
            assert sampling_noise.shape[1] == self.num_timesteps - 1
        if if_interpolate:
            return self._p_sample_loop_interpolate(shape, x_cond, start_noise, sampling_noise,
                                                   return_sampling_noise, return_timages,
                                                   noise2interpolate, interpolation_kwargs, clip)
        if self.self_condition:
            raise NotImplementedError("self_condition=True is not supported by the sampling engine")
        if seed is None and (start_noise is None or sampling_noise is None):
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())  # fixed, so a re-run draws the same noise

        # no host-side range check: a split-f16 tile whose operands leave the f16 range is
        # recomputed on exact-f32 MFMA inside the kernel (engine.py, exact_tile_f32)
        res = self.engine.sample_loop(shape[0], x_cond=x_cond, start_noise=start_noise,
                                      sampling_noise=sampling_noise,
                                      record=(return_sampling_noise, return_timages), seed=seed, row0=row0,
                                      out=out, clip=clip)
        img, start, noise_t, mean_t, imgs = res
        noise = start
        if return_sampling_noise:
            noise = (start, noise_t, imgs) if return_timages else (start, noise_t, mean_t)
        elif return_timages:
            noise = (start, imgs)
        return img, noise

    def _p_sample_loop_interpolate(self, shape, x_cond, start_noise, sampling_noise, return_sampling_noise,
                                   return_timages, noise2interpolate, interpolation_kwargs, clip=True):
        img = start_noise if start_noise is not None else self.get_start_noise(shape, device=self.betas.device)
        noise = img.clone()
        noise_t, mean_t, imgs = [], [], []
        for t in reversed(range(self.num_timesteps)):
            img, _, nt, mean = self.p_sample(img, t, None, clip_denoised=clip, sampling_noise=sampling_noise,
                                             x_cond=x_cond, if_interpolate=True, noise2interpolate=noise2interpolate,
                                             interpolation_kwargs=interpolation_kwargs)
            if t != 0:
                noise_t.append(nt)
                mean_t.append(mean)
                imgs.append(img)
        if return_sampling_noise:
            noise = (noise, torch.stack(noise_t, 1), torch.stack(imgs, 1) if return_timages else torch.stack(mean_t, 1))
        elif return_timages:
            noise = (noise, torch.stack(imgs, 1))
        return img, noise

    @torch.no_grad()
    def ddim_sample(self, shape, clip_denoised=True, x_cond=None, start_noise=None):
        # The reference's DDIM branch reads `times` before assignment (base.py:396) and can
        # never run; it is selected only when sampling_timesteps < timesteps.
        raise NotImplementedError("ddim_sample is broken in the reference (base.py:396) and not provided")

    @torch.no_grad()
    def sample(self, batch_size=16, *args, **kwargs):
        fn = self.p_sample_loop if not self.is_ddim_sampling else self.ddim_sample
        return fn((batch_size, self.channels, self.seq_length), *args, **kwargs)
