"""The CPU oracle against the reference's own outputs on the reference options pinned in round 6
(tests/golden/gen_golden.py gen_iso_paths / gen_noclip_release / gen_options):

* the isotropic pred_noise / pred_v objectives on the paths that go through p_mean_variance ->
  model_predictions (noise interpolation, direct p_mean_variance calls; base.py:219-241, 314-322);
* p_sample's clip_denoised=False (base.py:318-319 skipped), through sample()'s **kwargs;
* the config-selectable covariance / schedule options: diffusion_covariance_type='anisotropic',
  gamma_scheduler='mono_decrease', beta_schedule 'linear' / 'exp' (nonisotropic.py:36-68,
  base.py:39-61; configs/config_train_diffusion/model/skeleton_diffusion.yaml:42-44);
* the Denoiser's norm_type='layer' (Block: LayerNorm over the node axis, attention.py:19-28, 49-75).

The GPU side of the same fixtures is tests/test_gpu_options.py."""
import numpy as np
import pytest
import torch

import oracle as O
from conftest import (ISO_OBJECTIVES, LAYERNORM_MODELS, OPTION_CASES, WEIGHT_SEED, golden, interpolate_funct,
                      iso_path_inputs, layernorm_case, option_buffers, option_inputs, tol_rel)


@pytest.mark.parametrize("obj", ISO_OBJECTIVES)
@pytest.mark.parametrize("act", ["identity", "tanh"])
def test_oracle_iso_interpolation_and_p_mean_variance(obj, act):
    z = golden("iso_paths_T10")
    cfg = O.readme_config()
    sd = O.synthetic_state_dict(cfg, WEIGHT_SEED)
    bufs = O.isotropic_buffers(O.beta_schedule("cosine", 10), objective=obj)
    start, samp, noise2 = iso_path_inputs()
    k = f"{obj}_{act}"
    kw = dict(isotropic=True, activation=act, objective=obj)
    img, means = O.p_sample_loop(sd, cfg, bufs, start, samp, record_means=True, noise2interpolate=noise2,
                                 interpolate_funct=interpolate_funct, **kw)
    steps = z["mean_t_steps"]
    np.testing.assert_allclose(img.numpy(), z[f"{k}_interp_img"], atol=2e-5, rtol=0)
    np.testing.assert_allclose(means[:, steps].numpy(), z[f"{k}_interp_mean_t"], atol=2e-5, rtol=0)
    t = int(z["pmv_t"])
    for c in ("clip", "noclip"):
        mean, var, lv, x0 = O.p_mean_variance(sd, cfg, bufs, start, t, clip=(c == "clip"), **kw)
        for name, v in (("mean", mean), ("x0", x0), ("var", var), ("logvar", lv)):
            ref = z[f"{k}_pmv_{c}_{name}"]
            assert v.shape == ref.shape, (name, v.shape, ref.shape)
            np.testing.assert_allclose(v.numpy(), ref, atol=tol_rel(ref, 2e-5), rtol=0, err_msg=f"{c} {name}")
    img, means = O.p_sample_loop(sd, cfg, bufs, start, samp, record_means=True, clip=False, **kw)
    np.testing.assert_allclose(img.numpy(), z[f"{k}_noclip_img"], atol=tol_rel(z[f"{k}_noclip_img"], 2e-5), rtol=0)
    np.testing.assert_allclose(means[:, steps].numpy(), z[f"{k}_noclip_mean_t"],
                               atol=tol_rel(z[f"{k}_noclip_mean_t"], 2e-5), rtol=0)
    if obj != "pred_x0":  # the objective's x0 conversion is what the interpolation path needed
        assert np.abs(z[f"{k}_pmv_noclip_x0"]).max() > 1.0


def test_oracle_release_no_clip():
    z = golden("noclip_h36m16_T10")
    cfg = O.release_config(16, z["node_types"])
    sd = O.synthetic_state_dict(cfg, WEIGHT_SEED, float(z["final_scale"]))
    from conftest import pinned_cov, variant_inputs
    S, L, U = pinned_cov(16)
    bufs = O.nonisotropic_buffers(S, L, U, O.beta_schedule("cosine", 10))
    xc, start, samp, noise2 = variant_inputs(z)
    img, means = O.p_sample_loop(sd, cfg, bufs, start, samp, x_cond=xc, record_means=True, clip=False)
    np.testing.assert_allclose(img.numpy(), z["img"], atol=1e-6, rtol=0)
    np.testing.assert_allclose(means.numpy(), z["mean_t"], atol=1e-6, rtol=0)
    assert np.abs(z["img"]).max() > 1.0  # unclamped x0 reached the output
    img, _ = O.p_sample_loop(sd, cfg, bufs, start, samp, x_cond=xc, clip=False, noise2interpolate=noise2,
                             interpolate_funct=interpolate_funct)
    np.testing.assert_allclose(img.numpy(), z["interp_img"], atol=1e-6, rtol=0)
    t = int(z["step_t"])
    mean, _, lv, x0 = O.p_mean_variance(sd, cfg, bufs, start, t, x_cond=xc, clip=False)
    np.testing.assert_allclose(x0.numpy(), z["step_x0"], atol=1e-6, rtol=0)
    np.testing.assert_allclose(mean.numpy(), z["step_mean"], atol=1e-6, rtol=0)
    x = mean + bufs["U"] @ ((0.5 * lv).exp() * samp[:, samp.shape[1] - t])
    np.testing.assert_allclose(x.numpy(), z["step_x"], atol=1e-6, rtol=0)


@pytest.mark.parametrize("name", list(OPTION_CASES))
@pytest.mark.parametrize("model", ["readme", "release"])
def test_oracle_diffusion_options(name, model):
    """Every diffusion buffer of the option (the oracle's restatement of nonisotropic.py:36-127
    and base.py:39-61 on the reference's own Sigma_N / Lambda_N / U) and the sampled chain."""
    z = golden(f"option_{name}")
    S, L, U = (torch.from_numpy(z[f"{model}_buf_{k}"]) for k in ("Sigma_N", "Lambda_N", "U"))
    bufs = option_buffers(name, S, L, U)
    Tn = int(z["num_timesteps"])
    assert bufs["betas"].shape[0] == Tn
    for k, v in bufs.items():
        np.testing.assert_allclose(v.numpy(), z[f"{model}_buf_{k}"], atol=tol_rel(z[f"{model}_buf_{k}"], 1e-6),
                                   rtol=0, err_msg=k)
    cfg, sd, xc, start, samp = option_inputs(z, model)
    img, means = O.p_sample_loop(sd, cfg, bufs, start, samp, x_cond=xc, record_means=True)
    np.testing.assert_allclose(img.numpy(), z[f"{model}_img"], atol=1e-6, rtol=0)
    np.testing.assert_allclose(means[:, z["mean_t_steps"]].numpy(), z[f"{model}_mean_t"], atol=1e-6, rtol=0)


def test_options_change_the_chain():
    """Each option's chain differs from the default (cosine, skeleton-diffusion) chain's: the fixture
    exercises the option, not a no-op."""
    base = golden("option_anisotropic")  # release chains share their inputs across the option files
    for name in OPTION_CASES:
        z = golden(f"option_{name}")
        for other in OPTION_CASES:
            if other != name:
                assert np.abs(z["release_img"] - golden(f"option_{other}")["release_img"]).max() > 1e-4
    assert base["num_timesteps"] == 10 and golden("option_exp")["num_timesteps"] == 11


@pytest.mark.parametrize("name", list(OPTION_CASES))
def test_product_buffers_of_options(name):
    """The product module's 18 diffusion buffers (host setup, core/diffusion/) under each option equal
    the reference's (the plan is built from them)."""
    from conftest import build_option_diffusion

    z = golden(f"option_{name}")
    for model in ("readme", "release"):
        d = build_option_diffusion(name, model, z)
        assert d.num_timesteps == int(z["num_timesteps"])
        for k, v in d.state_dict().items():
            if k.startswith("model."):
                continue
            ref = z[f"{model}_buf_{k}"]
            np.testing.assert_allclose(v.numpy(), ref, atol=tol_rel(ref, 1e-6), rtol=0, err_msg=f"{model} {k}")


@pytest.mark.parametrize("model", LAYERNORM_MODELS)
def test_oracle_layernorm_denoiser(model):
    """norm_type='layer': the Denoiser forward at t = 3 and the sampled T = 10 chain (README J = 16,
    release H36M J = 16, release AMASS J = 21)."""
    z = golden("layernorm_T10")
    cfg, sd, xc, start, samp, bufs = layernorm_case(model, z)
    t = torch.full((start.shape[0],), int(z["fwd_t"]), dtype=torch.long)
    out = O.denoiser_forward(sd, cfg, start, t, xc)
    np.testing.assert_allclose(out.numpy(), z[f"{model}_fwd"], atol=2e-6, rtol=0)
    img, means = O.p_sample_loop(sd, cfg, bufs, start, samp, x_cond=xc, record_means=True)
    np.testing.assert_allclose(img.numpy(), z[f"{model}_img"], atol=2e-6, rtol=0)
    np.testing.assert_allclose(means.numpy(), z[f"{model}_mean_t"], atol=2e-6, rtol=0)
    # the norm is exercised: the same weights without it give another output
    import dataclasses
    plain = {k: v for k, v in sd.items() if ".norm.norm." not in k}
    other = O.denoiser_forward(plain, dataclasses.replace(cfg, norm_type="none"), start, t, xc)
    assert (other - out).abs().max() > 1e-2


def test_product_module_layernorm_forward():
    """The product Denoiser module (torch path, core/network/layers.py) with norm_type='layer'
    reproduces the reference's forward."""
    from conftest import build_layernorm_diffusion

    z = golden("layernorm_T10")
    for model in LAYERNORM_MODELS:
        d = build_layernorm_diffusion(model, z)
        _, _, xc, start, _, _ = layernorm_case(model, z)
        t = torch.full((start.shape[0],), int(z["fwd_t"]), dtype=torch.long)
        with torch.no_grad():
            out = d.model(start, t, None, xc)
        np.testing.assert_allclose(out.numpy(), z[f"{model}_fwd"], atol=2e-6, rtol=0, err_msg=model)
