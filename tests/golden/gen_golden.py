#!/usr/bin/env python3
"""Generate the golden parity fixtures by running the REFERENCE itself on CPU.

Build-container tool only: it imports the read-only reference tree at /root/reference
(which does not exist on the GPU box) and writes small .npz fixtures next to this file.
Only inputs-by-seed and reference outputs are written; weights are regenerated from a seed
by `skeletondiffusion_amd.synthetic` wherever the fixtures are consumed.

Third-party gap: the reference's Denoiser imports
`denoising_diffusion_pytorch.denoising_diffusion_pytorch_1d.{SinusoidalPosEmb,
RandomOrLearnedSinusoidalPosEmb}` (pinned `denoising_diffusion_pytorch==1.9.4`,
reference README.md:151), which is not installed here.  The module below is a restatement of
that package's published sinusoidal embedding:
    half = dim // 2; f_k = exp(-k * ln(theta) / (half - 1)), k < half
    emb(t) = cat(sin(t * f), cos(t * f))
It is injected into sys.modules for the duration of this script; nothing of the reference is
copied into the repository.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py [metrics]
"""
from __future__ import annotations

import math
import os
import sys
import types

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True

import numpy as np
import torch
from torch import nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("SKELDIFF_REFERENCE", "/root/reference")
sys.path.insert(0, REPO)

from skeletondiffusion_amd import synthetic  # noqa: E402


def _install_ddp_shim() -> None:
    class SinusoidalPosEmb(nn.Module):
        def __init__(self, dim, theta=10000):
            super().__init__()
            self.dim = dim
            self.theta = theta

        def forward(self, x):
            half = self.dim // 2
            scale = math.log(self.theta) / (half - 1)
            freqs = torch.exp(torch.arange(half, device=x.device) * -scale)
            arg = x[:, None] * freqs[None, :]
            return torch.cat((arg.sin(), arg.cos()), dim=-1)

    class RandomOrLearnedSinusoidalPosEmb(nn.Module):
        def __init__(self, dim, is_random=False):
            super().__init__()
            assert dim % 2 == 0
            self.weights = nn.Parameter(torch.randn(dim // 2), requires_grad=not is_random)

        def forward(self, x):
            x = x[:, None]
            freqs = x * self.weights[None, :] * 2 * math.pi
            fouriered = torch.cat((freqs.sin(), freqs.cos()), dim=-1)
            return torch.cat((x, fouriered), dim=-1)

    pkg = types.ModuleType("denoising_diffusion_pytorch")
    sub = types.ModuleType("denoising_diffusion_pytorch.denoising_diffusion_pytorch_1d")
    sub.SinusoidalPosEmb = SinusoidalPosEmb
    sub.RandomOrLearnedSinusoidalPosEmb = RandomOrLearnedSinusoidalPosEmb
    pkg.denoising_diffusion_pytorch_1d = sub
    pkg.__version__ = "1.9.4-restated"
    sys.modules["denoising_diffusion_pytorch"] = pkg
    sys.modules["denoising_diffusion_pytorch.denoising_diffusion_pytorch_1d"] = sub


_install_ddp_shim()
sys.path.insert(0, REF)
from src.core.diffusion import (  # noqa: E402
    IsotropicGaussianDiffusion, NonisotropicGaussianDiffusion, get_cov_from_corr)
from src.core.network import Denoiser  # noqa: E402
from src.data.skeleton.kinematic import (  # noqa: E402
    AMASSKinematic, FreeManKinematic, H36MKinematic)

torch.set_num_threads(8)
torch.use_deterministic_algorithms(True)

# -------------------------------------------------------------------------------------------
# skeletons (hip excluded, as in eval: configs/config_eval/task/hmp.yaml:4)
SKELETONS = {
    "h36m16": lambda: H36MKinematic(num_joints=17, if_consider_hip=False),
    "amass21": lambda: AMASSKinematic(num_joints=22, if_consider_hip=False),
    "mano51": lambda: AMASSKinematic(num_joints=52, if_consider_hip=False),
    "freeman17": lambda: FreeManKinematic(if_consider_hip=False),
    # hip-included AMASS-MANO (amass.py:81-83): the root joint is a node (config 3's J=52 label)
    # (the compound skeleton class takes node_hip from motion/base.py:5, `Skeleton.node_hip`)
    "mano52": lambda: type("AMASSKinematicHip", (AMASSKinematic,), {"node_hip": {0: "GlobalRoot"}})(
        num_joints=52, if_consider_hip=True),
}

RELEASE_ARCH = dict(use_attention=True, self_condition=False, norm_type="none", depth=4,
                    attn_dim_head=32, attn_heads=8, learn_influence=True)

WEIGHT_SEED = 1234


def _save(name: str, **arrays) -> None:
    path = os.path.join(HERE, name + ".npz")
    clean = {}
    for k, v in arrays.items():
        if torch.is_tensor(v):
            v = v.detach().cpu().numpy()
        clean[k] = np.asarray(v)
    np.savez_compressed(path, **clean)
    print(f"wrote {path}: {os.path.getsize(path) / 1024:.1f} KiB")


def diffusion_buffers(diff) -> dict:
    return {f"buf_{k}": v for k, v in diff.state_dict().items() if not k.startswith("model.")}


def build_release(skel_key, T, seed=WEIGHT_SEED, final_scale=1.0, arch=None, **diff_kw):
    sk = SKELETONS[skel_key]()
    J = sk.num_nodes
    node_types = sk.nodes_type_id
    corr = sk.adj_matrix
    model = Denoiser(dim=96, cond_dim=96, out_dim=96, channels=J, num_nodes=J,
                     node_types=node_types, **dict(RELEASE_ARCH, **(arch or {})))
    synthetic.fill_module_(model, seed)
    if final_scale != 1.0:  # push x0 past +-1 so the clamp (base.py:318-319) is exercised
        with torch.no_grad():
            model.final_glin.weight.mul_(final_scale)
            model.final_glin.bias.mul_(final_scale)
    Sigma_N, Lambda_N, U = get_cov_from_corr(correlation_matrix=corr, if_sigma_n_scale=True,
                                             sigma_n_scale="spectral", if_run_as_isotropic=False)
    kw = dict(beta_schedule="cosine", diffusion_covariance_type="skeleton-diffusion", gamma_scheduler="cosine",
              loss_reduction_type="l1")
    kw.update(diff_kw)
    diff = NonisotropicGaussianDiffusion(Sigma_N=Sigma_N, Lambda_N=Lambda_N, U=U, model=model,
                                         latent_size=96, diffusion_timesteps=T,
                                         diffusion_objective="pred_x0",
                                         diffusion_conditioning=True, **kw)
    diff.eval()
    return sk, corr, node_types, diff


def capture_forward(model, x, t, x_cond):
    acts = {}
    hooks = []

    def hook(name):
        def f(_m, _i, out):
            acts[name] = out.detach().clone()
        return f

    hooks.append(model.init_lin.register_forward_hook(hook("init_lin")))
    for i, (res, attn) in enumerate(model.layers):
        hooks.append(res.register_forward_hook(hook(f"layer{i}_res")))
        hooks.append(attn.register_forward_hook(hook(f"layer{i}_attn")))
    hooks.append(model.final_res_block.register_forward_hook(hook("final_res")))
    with torch.no_grad():
        out = model(x, t, None, x_cond)
    for h in hooks:
        h.remove()
    return out, acts


def gen_covariances(keys=None):
    for key, ctor in SKELETONS.items():
        if keys and key not in keys:
            continue
        sk = ctor()
        corr = sk.adj_matrix
        Sigma_N, Lambda_N, U = get_cov_from_corr(correlation_matrix=corr, if_sigma_n_scale=True,
                                                 sigma_n_scale="spectral", if_run_as_isotropic=False)
        arrays = dict(corr=corr, node_types=sk.nodes_type_id, Sigma_N=Sigma_N, Lambda_N=Lambda_N, U=U,
                      node_names=np.array(list(sk.node_dict.values())))
        J = corr.shape[0]
        dummy = Denoiser(dim=96, cond_dim=0, out_dim=96, channels=J, num_nodes=J, depth=1)
        for T in (10, 100):
            d = NonisotropicGaussianDiffusion(Sigma_N=Sigma_N, Lambda_N=Lambda_N, U=U, model=dummy,
                                              diffusion_timesteps=T)
            for k, v in diffusion_buffers(d).items():
                if v.dim() == 3 and T == 100:
                    v = v[[0, 1, 50, 99]]  # keep the fixtures small at T=100
                arrays[f"T{T}_{k}"] = v
        _save(f"cov_{key}", **arrays)


def gen_readme():
    """Config 1: README plug-and-play Denoiser (J=16, D=96, T=10), `README.md:72-97`."""
    J, B, T = 16, 4, 10
    corr = torch.from_numpy(synthetic.readme_correlation(J, seed=7))
    start = torch.from_numpy(synthetic.normal((B, J, 96), seed=11))
    samp = torch.from_numpy(synthetic.normal((B, T - 1, J, 96), seed=12))
    x_train = torch.from_numpy(synthetic.uniform((8, J, 96), seed=13, low=0.0, high=1.0))
    train_noise = torch.from_numpy(synthetic.normal((8, J, 96), seed=14))
    train_t = torch.tensor([0, 1, 2, 3, 5, 7, 8, 9])
    out = dict(corr=corr, train_t=train_t)
    for mode in ("noniso", "iso_as_noniso", "isotropic"):
        model = Denoiser(dim=96, cond_dim=0, out_dim=96, channels=J, num_nodes=J)
        synthetic.fill_module_(model, WEIGHT_SEED)
        if mode == "isotropic":
            diff = IsotropicGaussianDiffusion(model=model, diffusion_timesteps=T)
        else:
            Sigma_N, Lambda_N, U = get_cov_from_corr(correlation_matrix=corr, if_sigma_n_scale=True,
                                                     sigma_n_scale="spectral",
                                                     if_run_as_isotropic=(mode == "iso_as_noniso"))
            diff = NonisotropicGaussianDiffusion(Sigma_N=Sigma_N, Lambda_N=Lambda_N, U=U, model=model,
                                                 timesteps=10)
        diff.eval()
        with torch.no_grad():
            img, (noise0, noise_t, mean_t) = diff.sample(batch_size=B, start_noise=start.clone(),
                                                         sampling_noise=samp.clone(),
                                                         return_sampling_noise=True)
            loss, lw, mout = diff.p_losses(x_train.clone(), train_t, noise=train_noise.clone())
        out.update({f"{mode}_img": img, f"{mode}_mean_t": mean_t, f"{mode}_loss": loss,
                    f"{mode}_loss_weight": lw, f"{mode}_model_out": mout})
        for k, v in diffusion_buffers(diff).items():
            out[f"{mode}_{k}"] = v
    _save("readme16_T10", **out)


def gen_iso_objectives():
    """IsotropicGaussianDiffusion sampled with the pred_noise and pred_v objectives (x0 from
    predict_start_from_noise / _from_v, isotropic.py:48-70; base.py:219-241), README Denoiser,
    J=16, T=10, identity and tanh diffusion activation (round 5)."""
    J, B, T = 16, 4, 10
    start = torch.from_numpy(synthetic.normal((B, J, 96), seed=11))
    samp = torch.from_numpy(synthetic.normal((B, T - 1, J, 96), seed=12))
    out = {}
    for obj in ("pred_noise", "pred_v"):
        for act in ("identity", "tanh"):
            model = Denoiser(dim=96, cond_dim=0, out_dim=96, channels=J, num_nodes=J)
            synthetic.fill_module_(model, WEIGHT_SEED)
            diff = IsotropicGaussianDiffusion(model=model, diffusion_timesteps=T, diffusion_objective=obj,
                                              diffusion_activation=act).eval()
            with torch.no_grad():
                img, (noise0, noise_t, mean_t) = diff.sample(batch_size=B, start_noise=start.clone(),
                                                             sampling_noise=samp.clone(), return_sampling_noise=True)
            out[f"{obj}_{act}_img"] = img
            out[f"{obj}_{act}_mean_t"] = mean_t
    out["start"], out["samp"] = start, samp
    _save("iso_objectives_T10", **out)


def gen_release(skel_key, T, B_seq, futures, with_acts, steps_to_keep=None, tag=None,
                final_scale=1.0):
    sk, corr, node_types, diff = build_release(skel_key, T, final_scale=final_scale)
    J = corr.shape[0]
    B = B_seq * futures
    x_cond_seq = torch.from_numpy(synthetic.uniform((B_seq, J, 96), seed=21))
    start = torch.from_numpy(synthetic.normal((B, J, 96), seed=22))
    samp = torch.from_numpy(synthetic.normal((B, T - 1, J, 96), seed=23))
    x_cond = x_cond_seq.repeat_interleave(futures, 0)
    with torch.no_grad():
        img, (noise0, noise_t, mean_t) = diff.sample(batch_size=B, x_cond=x_cond,
                                                     start_noise=start.clone(),
                                                     sampling_noise=samp.clone(),
                                                     return_sampling_noise=True)
    out = dict(img=img, node_types=node_types, corr=corr, B_seq=B_seq, futures=futures, T=T,
               final_scale=final_scale, weight_seed=WEIGHT_SEED)
    if steps_to_keep is None:
        out["mean_t"] = mean_t
    else:
        out["mean_t_steps"] = np.array(steps_to_keep)
        out["mean_t"] = mean_t[:, steps_to_keep]
    if with_acts:
        tt = torch.full((B,), T - 1, dtype=torch.long)
        x0, acts = capture_forward(diff.model, start.clone(), tt, x_cond)
        out["fwd_t"] = T - 1
        out["fwd_x0"] = x0
        for k, v in acts.items():
            out[f"act_{k}"] = v
        # training path: p_losses at fixed t / noise
        t_train = torch.arange(B) % T
        train_noise = torch.from_numpy(synthetic.normal((B, J, 96), seed=24))
        x_start = torch.from_numpy(synthetic.uniform((B, J, 96), seed=25))
        loss, lw, mout = diff.p_losses(x_start.clone(), t_train, noise=train_noise.clone(), x_cond=x_cond)
        out.update(train_t=t_train, train_loss=loss.detach(), train_loss_weight=lw,
                   train_model_out=mout.detach())
    _save(tag or f"release_{skel_key}_T{T}", **out)


INTERP_W = (0.25, 0.75)  # interpolate_funct(n1, n2) = 0.25 n1 + 0.75 n2 (consumers restate it)


def gen_variants():
    """Optional sample() surface on the release H36M J=16 Denoiser, T=10, 1 sequence x 3 futures:
    Denoiser(use_attention=False) (generator.py:65: Residual(PreNorm(StaticGraphLinear))),
    diffusion_activation='tanh' (base.py:78-79, 254), return_timages (base.py:371-389) and noise
    interpolation (base.py:335-338, nonisotropic.py:218-227) with a fixed interpolate_funct."""
    T, B_seq, futures = 10, 1, 3
    B = B_seq * futures
    out = {"B_seq": B_seq, "futures": futures, "T": T}
    x_cond = torch.from_numpy(synthetic.uniform((B_seq, 16, 96), seed=21)).repeat_interleave(futures, 0)
    start = torch.from_numpy(synthetic.normal((B, 16, 96), seed=22))
    samp = torch.from_numpy(synthetic.normal((B, T - 1, 16, 96), seed=23))
    noise2 = torch.from_numpy(synthetic.normal((B, T - 1, 16, 96), seed=26))
    cases = {
        "noattn": dict(arch=dict(use_attention=False)),
        "tanh": dict(final_scale=8.0, diffusion_activation="tanh"),
        "base": {},
    }
    for name, kw in cases.items():
        _, corr, node_types, diff = build_release("h36m16", T, **kw)
        out["node_types"], out["corr"] = node_types, corr
        with torch.no_grad():
            img, (_, _, mean_t) = diff.sample(batch_size=B, x_cond=x_cond, start_noise=start.clone(),
                                              sampling_noise=samp.clone(), return_sampling_noise=True)
            out[f"{name}_img"], out[f"{name}_mean_t"] = img, mean_t
            if name == "base":
                img2, (_, timgs) = diff.sample(batch_size=B, x_cond=x_cond, start_noise=start.clone(),
                                               sampling_noise=samp.clone(), return_timages=True)
                out["timages_img"], out["timages"] = img2, timgs
                a, b = INTERP_W
                img3, _ = diff.sample(batch_size=B, x_cond=x_cond, start_noise=start.clone(),
                                      sampling_noise=samp.clone(), if_interpolate=True,
                                      noise2interpolate=noise2.clone(),
                                      interpolation_kwargs={"interpolate_funct": lambda n1, n2: a * n1 + b * n2})
                out["interp_img"] = img3
        if name == "noattn":
            out["noattn_keys"] = np.array(sorted(diff.state_dict().keys()))
    _save("variants_h36m16_T10", **out)


def gen_new_r02():
    """Round-2 fixtures: BASELINE config 3 at T=100 (MANO J=51) and config 4 at T=1000 (H36M
    J=16), plus the optional sample() surface (gen_variants)."""
    gen_variants()
    gen_release("mano51", 100, B_seq=2, futures=2, with_acts=False, steps_to_keep=[0, 9, 49, 98])
    gen_release("h36m16", 1000, B_seq=1, futures=2, with_acts=False,
                steps_to_keep=[0, 1, 2, 3, 4, 499, 994, 995, 996, 997, 998])


def gen_hip_included():
    """Round 2: the hip-included MANO skeleton (J = 52, if_consider_hip=True): covariances and a
    T = 10 release sample (1 sequence x 2 futures)."""
    gen_covariances(["mano52"])
    gen_release("mano52", 10, B_seq=1, futures=2, with_acts=False)


def gen_new_r03():
    """Round 3: config 3's hip-included label (MANO J = 52) at the benched T = 100, 2 sequences x
    2 futures, posterior means of four steps kept."""
    gen_release("mano52", 100, B_seq=2, futures=2, with_acts=False, steps_to_keep=[0, 9, 49, 98])


def gen_metrics():
    """The reference's multimodal metrics (src/metrics/multimodal.py) on synthetic samples: latent
    APD (L1) and APD (L2) over 50 futures of (J=16, 96) latents, and ADE / FDE of (frames, J*3)
    motions against a target, incl. the per-sample (reduction != 'mean') form."""
    from src.metrics.multimodal import ade, apd, fde, lat_apd, mmade, mmfde

    lat = torch.from_numpy(synthetic.normal((3, 50, 16, 96), seed=31)) * 0.3
    motion = torch.from_numpy(synthetic.normal((2, 7, 20, 16, 3), seed=32))  # (B, S, T, J, 3)
    target = torch.from_numpy(synthetic.normal((2, 20, 16, 3), seed=33))
    # inputs are regenerated from the seeds by the consumers (tests/test_metrics*.py)
    _save("metrics", lat_apd=lat_apd(lat), lat_apd_l2=apd(lat.unsqueeze(2)),
          apd=apd(motion), ade=ade(target, motion), fde=fde(target, motion),
          ade_per_sample=ade(target, motion, reduction="none"), fde_per_sample=fde(target, motion, reduction="none"),
          ade_t5_15=ade(target, motion, t0=5, t=15), apd_t5_15=apd(motion, t0=5, t=15),
          **gen_mm(motion, target, mmade, mmfde))


def mm_inputs():
    """Multimodal ground truths for the 3 sequences of mm_motion: 3, 1 and 2 of them (ragged)."""
    motion = torch.from_numpy(synthetic.normal((3, 7, 20, 16, 3), seed=34))
    gts = torch.from_numpy(synthetic.normal((4, 20, 16, 3), seed=35))
    target = torch.from_numpy(synthetic.normal((3, 20, 16, 3), seed=36))  # sliced, otherwise unused
    return motion, [gts[:3], gts[3:4], gts[1:3]], target


def gen_mm(motion, target, mmade, mmfde):
    mm_motion, mm_gt, mm_target = mm_inputs()
    try:  # a sequence without ground truths: the reference's reshape raises
        mmade(mm_target, mm_motion, [mm_gt[0], mm_gt[1], mm_gt[2][:0]])
        empty_raises = False
    except RuntimeError:
        empty_raises = True
    return dict(mmade=mmade(mm_target, mm_motion, mm_gt), mmfde=mmfde(mm_target, mm_motion, mm_gt),
                mmade_t5_15=mmade(mm_target, mm_motion, mm_gt, t0=5, t=15), mm_empty_raises=empty_raises)


AE_KW = dict(num_nodes=16, encoder_hidden_size=96, decoder_hidden_size=96, latent_size=96, input_size=3,
             z_activation="tanh", enc_num_layers=1, output_size=3, recurrent_arch_enc="StaticGraphGRU",
             recurrent_arch_decoder="StaticGraphGRU", if_consider_hip=False)
AE_SEED = 4321


def gen_decoder():
    """The reference's AutoEncoder (src/core/network/nn/autoencoder.py, release autoencoder.yaml
    sizes, H36M 16-joint node types) with synthetic weights: the encoder's past embedding of 3
    observed sequences, and AutoEncoder.decode of 3 x 4 sampled latents for 120 frames."""
    from src.core.network.nn.autoencoder import AutoEncoder
    from skeletondiffusion_amd.skeletons import skeleton

    _, _, _, types = skeleton("h36m16")
    m = AutoEncoder(node_types=torch.from_numpy(types), **AE_KW).eval()
    synthetic.fill_module_(m, AE_SEED)
    past = torch.from_numpy(synthetic.normal((3, 30, 16, 3), seed=41)) * 0.3
    lat = torch.from_numpy(synthetic.uniform((12, 16, 96), seed=42))
    with torch.no_grad():
        z_past = m.get_past_embedding(past)
        out = m.decode(past.repeat_interleave(4, 0), lat, z_past.repeat_interleave(4, 0), ph=120)
    _save("decoder", out=out, z_past=z_past, keys=np.array(sorted(m.state_dict().keys())))


def gen_best_of_k():
    """The best-of-k training relaxation with the reference's modules: the release
    H36M Denoiser's p_losses with n_train_samples = k (base.py:262-300; fixed t and noise), the
    reference AutoEncoder's decode of the k sampled x0 per sequence and AutoEncoder.loss(reduction=
    'none') against the future (autoencoder.py:80-98) -- the input_space similarity of the release
    configs -- and the selection of trainer.py:218-220 (`min(axis=-1).indices` + `torch.gather`,
    restated: trainer.py imports ignite, absent here).  Also AutoEncoder.loss alone on random poses,
    l1 and mse."""
    from src.core.network.nn.autoencoder import AutoEncoder

    _, _, node_types, diff = build_release("h36m16", 10)
    ae = AutoEncoder(node_types=torch.as_tensor(node_types), **AE_KW).eval()
    synthetic.fill_module_(ae, AE_SEED)
    b, k, ph = 3, 4, 12
    data = torch.from_numpy(synthetic.uniform((b, 16, 96), seed=61))
    x_cond = torch.from_numpy(synthetic.uniform((b, 16, 96), seed=62))
    t = torch.tensor([1, 5, 9])
    noise = torch.from_numpy(synthetic.normal((b * k, 16, 96), seed=63))
    past = torch.from_numpy(synthetic.normal((b, 30, 16, 3), seed=64)) * 0.3
    loss, w, samples = diff.p_losses(data, t, noise=noise, x_cond=x_cond, n_train_samples=k)
    with torch.no_grad():
        xc = x_cond.repeat_interleave(k, dim=0)
        out = ae.decode(past.repeat_interleave(k, dim=0), samples, xc, ph).view(b, k, ph, 16, 3)
        # the future: a perturbed copy of one decoded sample per sequence (2, 0, 3), so the
        # closest sample is decided by a margin well above the fp32 / HIP-decoder error
        fut = out[torch.arange(b), torch.tensor([2, 0, 3])] + \
            torch.from_numpy(synthetic.normal((b, ph, 16, 3), seed=65)) * 1e-4
        sim = ae.loss(out, fut.unsqueeze(1).repeat_interleave(k, dim=1), reduction="none")
        idx = sim.view(b, -1).min(axis=-1).indices
        idx_latent = loss.detach().view(b, -1).min(axis=-1).indices
    sel = torch.gather(loss.view(b, -1), dim=1, index=idx.unsqueeze(1)).squeeze(-1)
    final = (sel * w).mean()
    pred = torch.from_numpy(synthetic.normal((2, 5, 7, 21, 3), seed=66))
    tgt = torch.from_numpy(synthetic.normal((2, 7, 21, 3), seed=67))
    ns = types.SimpleNamespace
    pl1 = AutoEncoder.loss(ns(loss_pose_type="l1"), pred, tgt.unsqueeze(1).repeat_interleave(5, dim=1), reduction="none")
    pmse = AutoEncoder.loss(ns(loss_pose_type="mse"), pred, tgt.unsqueeze(1).repeat_interleave(5, dim=1),
                            reduction="none")
    _save("best_of_k", data=data, x_cond=x_cond, t=t, noise=noise, past=past, fut=fut, k=k, ph=ph,
          loss=loss.detach(), weight=w, samples=samples.detach(), decoded=out, sim=sim, idx=idx,
          idx_latent=idx_latent, sel=sel.detach(), final=final.detach(), pose_pred=pred, pose_target=tgt,
          pose_l1=pl1, pose_mse=pmse)


def gen_best_of_k_metric():
    """Best-of-k in `metric_space` (trainer.py:193-198 + 213-214) on the fixture gen_best_of_k wrote:
    the reference skeleton of the release task config (SkeletonRescalePose, if_consider_hip False,
    pose_box_size 1.5: configs/config_train_autoencoder/task/hmp.yaml) maps the decoded samples and
    the future to metric space; the similarity is the per-sample L2 over the flattened joints, mean
    over frames; the selection is trainer.py:218-220 (restated: trainer.py imports ignite, absent)."""
    from src.data.skeleton.motion.rescalepose import SkeletonRescalePose

    z = np.load(os.path.join(HERE, "best_of_k.npz"))
    sk = SkeletonRescalePose(if_consider_hip=False, pose_box_size=1.5, obs_length=30, pred_length=int(z["ph"]))
    out, fut = torch.from_numpy(z["decoded"]), torch.from_numpy(z["fut"])
    loss = torch.from_numpy(z["loss"])
    b, k = out.shape[:2]
    out_c = sk.transform_to_metric_space(out).flatten(start_dim=3)
    fut_c = sk.transform_to_metric_space(fut).unsqueeze(1).flatten(start_dim=3).repeat_interleave(k, dim=1)
    sim = torch.linalg.norm(out_c - fut_c, axis=-1).mean(axis=-1)
    idx = sim.view(b, -1).min(axis=-1).indices
    sel = torch.gather(loss.view(b, -1), dim=1, index=idx.unsqueeze(1)).squeeze(-1)
    _save("best_of_k_metric", out_c=out_c, fut_c=fut_c, sim=sim, idx=idx, sel=sel, pose_box_size=1.5)


def _interp(n1, n2):
    a, b = INTERP_W
    return a * n1 + b * n2


def gen_iso_paths():
    """Round 6: IsotropicGaussianDiffusion (README Denoiser, J=16, B=4, T=10) on the paths that go
    through p_mean_variance -> model_predictions (base.py:219-241, 314-322): noise interpolation
    (base.py:335-338, isotropic.py:97-103) for pred_x0 / pred_noise / pred_v x identity / tanh, one
    direct p_mean_variance call at t=6 with and without the clamp, and sample(clip_denoised=False)
    (the kwarg reaches p_sample through p_sample_loop's **kwargs, base.py:344,367)."""
    J, B, T = 16, 4, 10
    start = torch.from_numpy(synthetic.normal((B, J, 96), seed=11))
    samp = torch.from_numpy(synthetic.normal((B, T - 1, J, 96), seed=12))
    noise2 = torch.from_numpy(synthetic.normal((B, T - 1, J, 96), seed=13))
    keep = [0, 4, 8]  # mean_t steps kept (the inputs are regenerated from the seeds by the consumers)
    out = {"pmv_t": 6, "mean_t_steps": np.array(keep)}
    for obj in ("pred_x0", "pred_noise", "pred_v"):
        for act in ("identity", "tanh"):
            model = Denoiser(dim=96, cond_dim=0, out_dim=96, channels=J, num_nodes=J)
            synthetic.fill_module_(model, WEIGHT_SEED)
            diff = IsotropicGaussianDiffusion(model=model, diffusion_timesteps=T, diffusion_objective=obj,
                                              diffusion_activation=act).eval()
            k = f"{obj}_{act}"
            with torch.no_grad():
                img, (_, _, mean_t) = diff.sample(batch_size=B, start_noise=start.clone(), sampling_noise=samp.clone(),
                                                  return_sampling_noise=True, if_interpolate=True,
                                                  noise2interpolate=noise2.clone(),
                                                  interpolation_kwargs={"interpolate_funct": _interp})
                out[f"{k}_interp_img"], out[f"{k}_interp_mean_t"] = img, mean_t[:, keep]
                tt = torch.full((B,), 6, dtype=torch.long)
                for clip in (True, False):
                    mean, var, logvar, x0 = diff.p_mean_variance(start.clone(), tt, clip_denoised=clip)
                    c = "clip" if clip else "noclip"
                    out[f"{k}_pmv_{c}_mean"], out[f"{k}_pmv_{c}_x0"] = mean, x0
                    out[f"{k}_pmv_{c}_var"], out[f"{k}_pmv_{c}_logvar"] = var, logvar
                img, (_, _, mean_t) = diff.sample(batch_size=B, start_noise=start.clone(), sampling_noise=samp.clone(),
                                                  return_sampling_noise=True, clip_denoised=False)
                out[f"{k}_noclip_img"], out[f"{k}_noclip_mean_t"] = img, mean_t[:, keep]
    _save("iso_paths_T10", **out)


def gen_noclip_release():
    """Round 6: the release H36M J=16 sampler with clip_denoised=False (x0 pushed past +-1 by
    final_scale 8, so the missing clamp shows), plain and with noise interpolation, and one
    p_sample step (base.py:324-341 with clip_denoised=False) at t=4."""
    T, B_seq, futures = 10, 1, 3
    B = B_seq * futures
    _, corr, node_types, diff = build_release("h36m16", T, final_scale=8.0)
    x_cond = torch.from_numpy(synthetic.uniform((B_seq, 16, 96), seed=21)).repeat_interleave(futures, 0)
    start = torch.from_numpy(synthetic.normal((B, 16, 96), seed=22))
    samp = torch.from_numpy(synthetic.normal((B, T - 1, 16, 96), seed=23))
    noise2 = torch.from_numpy(synthetic.normal((B, T - 1, 16, 96), seed=26))
    out = {"B_seq": B_seq, "futures": futures, "T": T, "final_scale": 8.0, "node_types": node_types, "corr": corr}
    with torch.no_grad():
        img, (_, _, mean_t) = diff.sample(batch_size=B, x_cond=x_cond, start_noise=start.clone(),
                                          sampling_noise=samp.clone(), return_sampling_noise=True, clip_denoised=False)
        out["img"], out["mean_t"] = img, mean_t
        img, _ = diff.sample(batch_size=B, x_cond=x_cond, start_noise=start.clone(), sampling_noise=samp.clone(),
                             if_interpolate=True, noise2interpolate=noise2.clone(),
                             interpolation_kwargs={"interpolate_funct": _interp}, clip_denoised=False)
        out["interp_img"] = img
        x, x0, noise, mean = diff.p_sample(start.clone(), 4, None, clip_denoised=False, sampling_noise=samp.clone(),
                                           x_cond=x_cond)
        out.update(step_t=4, step_x=x, step_x0=x0, step_mean=mean)
    _save("noclip_h36m16_T10", **out)


# config-selectable diffusion options (configs/config_train_diffusion/model/skeleton_diffusion.yaml:42-44)
OPTION_CASES = {
    "anisotropic": dict(T=10, diff_kw=dict(diffusion_covariance_type="anisotropic")),
    "mono_decrease": dict(T=10, diff_kw=dict(gamma_scheduler="mono_decrease")),
    # linear at T=10 reaches beta = 2 (base.py:39-43 is not clipped): NaN buffers; T=100 ends at 0.2
    "linear": dict(T=100, diff_kw=dict(beta_schedule="linear")),
    "exp": dict(T=10, diff_kw=dict(beta_schedule="exp")),  # T+1 = 11 steps (base.py:57-61, 116)
}


def gen_options():
    """Round 6: the reference's config-selectable covariance / schedule options, each on the
    README Denoiser (J=16, B=4) and the release H36M J=16 Denoiser (2 sequences x 4 futures):
    every diffusion buffer and the sampled chain with supplied noise (nonisotropic.py:36-68,
    base.py:39-61,103-116)."""
    for name, case in OPTION_CASES.items():
        T, kw = case["T"], case["diff_kw"]
        out = {"T_arg": T}
        # README Denoiser, README correlation recipe
        J, B = 16, 4
        corr = torch.from_numpy(synthetic.readme_correlation(J, seed=7))
        model = Denoiser(dim=96, cond_dim=0, out_dim=96, channels=J, num_nodes=J)
        synthetic.fill_module_(model, WEIGHT_SEED)
        Sigma_N, Lambda_N, U = get_cov_from_corr(correlation_matrix=corr, if_sigma_n_scale=True,
                                                 sigma_n_scale="spectral", if_run_as_isotropic=False)
        diff = NonisotropicGaussianDiffusion(Sigma_N=Sigma_N, Lambda_N=Lambda_N, U=U, model=model,
                                             diffusion_timesteps=T, **kw).eval()
        Tn = diff.num_timesteps
        start = torch.from_numpy(synthetic.normal((B, J, 96), seed=11))
        samp = torch.from_numpy(synthetic.normal((B, Tn - 1, J, 96), seed=12))
        with torch.no_grad():
            img, (_, _, mean_t) = diff.sample(batch_size=B, start_noise=start.clone(), sampling_noise=samp.clone(),
                                              return_sampling_noise=True)
        keep = [0, 1, Tn // 2, Tn - 2]
        out.update(readme_corr=corr, readme_img=img, readme_mean_t=mean_t[:, keep], mean_t_steps=np.array(keep),
                   num_timesteps=Tn)
        for k, v in diffusion_buffers(diff).items():
            out[f"readme_{k}"] = v
        # release H36M
        sk, corr, node_types, diff = build_release("h36m16", T, **kw)
        bs, fu = 2, 4
        B = bs * fu
        x_cond = torch.from_numpy(synthetic.uniform((bs, 16, 96), seed=21))
        start = torch.from_numpy(synthetic.normal((B, 16, 96), seed=22))
        samp = torch.from_numpy(synthetic.normal((B, Tn - 1, 16, 96), seed=23))
        with torch.no_grad():
            img, (_, _, mean_t) = diff.sample(batch_size=B, x_cond=x_cond.repeat_interleave(fu, 0),
                                              start_noise=start.clone(), sampling_noise=samp.clone(),
                                              return_sampling_noise=True)
        out.update(release_img=img, release_mean_t=mean_t[:, keep], node_types=node_types, corr=corr,
                   B_seq=bs, futures=fu)
        for k, v in diffusion_buffers(diff).items():
            out[f"release_{k}"] = v
        _save(f"option_{name}", **out)


def gen_layernorm():
    """Round 6: the Denoiser with norm_type='layer' (Block: proj -> LayerNorm over the node axis ->
    FiLM -> tanh, attention.py:19-28, 49-75): README Denoiser (J=16, B=4, nonisotropic, README
    correlation) and the release H36M J=16 / AMASS J=21 Denoisers (2 sequences x 4 futures), T=10,
    supplied noise; one direct Denoiser forward at t=3 per model."""
    T = 10
    out = {"T": T, "fwd_t": 3}
    J, B = 16, 4
    corr = torch.from_numpy(synthetic.readme_correlation(J, seed=7))
    model = Denoiser(dim=96, cond_dim=0, out_dim=96, channels=J, num_nodes=J, norm_type="layer")
    synthetic.fill_module_(model, WEIGHT_SEED)
    Sigma_N, Lambda_N, U = get_cov_from_corr(correlation_matrix=corr, if_sigma_n_scale=True,
                                             sigma_n_scale="spectral", if_run_as_isotropic=False)
    diff = NonisotropicGaussianDiffusion(Sigma_N=Sigma_N, Lambda_N=Lambda_N, U=U, model=model,
                                         diffusion_timesteps=T).eval()
    start = torch.from_numpy(synthetic.normal((B, J, 96), seed=11))
    samp = torch.from_numpy(synthetic.normal((B, T - 1, J, 96), seed=12))
    with torch.no_grad():
        img, (_, _, mean_t) = diff.sample(batch_size=B, start_noise=start.clone(), sampling_noise=samp.clone(),
                                          return_sampling_noise=True)
        fwd = model(start.clone(), torch.full((B,), 3, dtype=torch.long))
    out.update(readme_corr=corr, readme_img=img, readme_mean_t=mean_t, readme_fwd=fwd)
    for k, v in diffusion_buffers(diff).items():
        out[f"readme_{k}"] = v
    for key in ("h36m16", "amass21"):
        sk, corr, node_types, diff = build_release(key, T, arch=dict(norm_type="layer"))
        J = corr.shape[0]
        bs, fu = 2, 4
        B = bs * fu
        x_cond = torch.from_numpy(synthetic.uniform((bs, J, 96), seed=21))
        start = torch.from_numpy(synthetic.normal((B, J, 96), seed=22))
        samp = torch.from_numpy(synthetic.normal((B, T - 1, J, 96), seed=23))
        with torch.no_grad():
            img, (_, _, mean_t) = diff.sample(batch_size=B, x_cond=x_cond.repeat_interleave(fu, 0),
                                              start_noise=start.clone(), sampling_noise=samp.clone(),
                                              return_sampling_noise=True)
            fwd = diff.model(start.clone(), torch.full((B,), 3, dtype=torch.long), None,
                             x_cond.repeat_interleave(fu, 0))
        out.update({f"{key}_img": img, f"{key}_mean_t": mean_t, f"{key}_fwd": fwd, f"{key}_node_types": node_types,
                    f"{key}_corr": corr})
    out.update(B_seq=2, futures=4)
    _save("layernorm_T10", **out)


def main():
    if sys.argv[1:] == ["layernorm"]:
        gen_layernorm()
        return
    if sys.argv[1:] == ["r06"]:
        gen_iso_paths()
        gen_noclip_release()
        gen_options()
        return
    if sys.argv[1:] == ["best_of_k_metric"]:
        gen_best_of_k_metric()
        return
    if sys.argv[1:] == ["iso_obj"]:
        gen_iso_objectives()
        return
    if sys.argv[1:] == ["best_of_k"]:
        gen_best_of_k()
        return
    if sys.argv[1:] == ["metrics"]:
        gen_metrics()
        return
    if sys.argv[1:] == ["decoder"]:
        gen_decoder()
        return
    if sys.argv[1:] == ["r02"]:
        gen_new_r02()
        return
    if sys.argv[1:] == ["hip"]:
        gen_hip_included()
        return
    if sys.argv[1:] == ["r03"]:
        gen_new_r03()
        return
    gen_metrics()
    gen_decoder()
    gen_covariances()
    gen_readme()
    gen_release("h36m16", 10, B_seq=2, futures=4, with_acts=True)
    gen_release("h36m16", 100, B_seq=2, futures=4, with_acts=False, steps_to_keep=[0, 9, 49, 98])
    gen_release("amass21", 10, B_seq=1, futures=4, with_acts=True, final_scale=8.0)
    gen_release("freeman17", 10, B_seq=1, futures=4, with_acts=False)
    gen_release("mano51", 10, B_seq=1, futures=2, with_acts=False)
    gen_new_r02()
    gen_hip_included()
    gen_new_r03()
    gen_best_of_k()
    gen_iso_objectives()
    gen_iso_paths()
    gen_noclip_release()
    gen_options()


if __name__ == "__main__":
    main()
