"""GPU parity on the reference options pinned in round 6 (the CPU oracle side is
tests/test_reference_options.py; fixtures from tests/golden/gen_golden.py, which ran the reference):

* IsotropicGaussianDiffusion pred_x0 / pred_noise / pred_v x identity / tanh on the paths through
  p_mean_variance -> model_predictions (noise interpolation, direct p_mean_variance calls;
  reference base.py:219-241, 314-341, isotropic.py:48-70, 97-103);
* clip_denoised=False (SD_FLAG_NO_CLIP: the update kernels skip the clamp), through sample()'s
  **kwargs as in the reference (base.py:344,367 -> :325), in eager and hipGraph mode;
* the config-selectable covariance / schedule options: anisotropic, mono_decrease, linear, exp
  (exp has T + 1 steps) on the README and the release Denoiser.

Tolerance: 1e-4 absolute (BASELINE.json north_star), scaled by the fixture's magnitude where the
unclamped pred_noise chains reach |x| ~ 1e3 (tol_rel)."""
import numpy as np
import pytest
import torch

from conftest import (ISO_OBJECTIVES, OPTION_CASES, WEIGHT_SEED, build_option_diffusion, build_release_diffusion,
                      golden, interpolate_funct, iso_path_inputs, tol_rel, variant_inputs)

pytestmark = pytest.mark.gpu
TOL = 1e-4


def _close(a, ref, tol=TOL):
    a = a.detach().float().cpu().numpy() if torch.is_tensor(a) else np.asarray(a)
    ref = np.asarray(ref)
    assert a.shape == ref.shape, (a.shape, ref.shape)
    err = float(np.abs(a - ref).max()) if a.size else 0.0
    assert err < tol_rel(ref, tol), (err, tol_rel(ref, tol))


def _iso(obj, act, cuda):
    from skeletondiffusion_amd import synthetic
    from skeletondiffusion_amd.core.diffusion import IsotropicGaussianDiffusion
    from skeletondiffusion_amd.core.network import Denoiser

    m = Denoiser(dim=96, cond_dim=0, out_dim=96, channels=16, num_nodes=16)
    synthetic.fill_module_(m, WEIGHT_SEED)
    return IsotropicGaussianDiffusion(model=m, diffusion_timesteps=10, diffusion_objective=obj,
                                      diffusion_activation=act).to(cuda).eval()


@pytest.mark.parametrize("obj", ISO_OBJECTIVES)
@pytest.mark.parametrize("act", ["identity", "tanh"])
def test_iso_objectives_interpolation_p_mean_variance_no_clip(obj, act, cuda):
    """the isotropic pred_noise / pred_v Denoiser output is converted to x0
    on the p_mean_variance path too (it fed the raw output in as x0 before round 6)."""
    z = golden("iso_paths_T10")
    d = _iso(obj, act, cuda)
    start, samp, noise2 = (t.to(cuda) for t in iso_path_inputs())
    k, steps = f"{obj}_{act}", z["mean_t_steps"]
    img, (_, _, mean_t) = d.sample(batch_size=4, start_noise=start, sampling_noise=samp, return_sampling_noise=True,
                                   if_interpolate=True, noise2interpolate=noise2,
                                   interpolation_kwargs={"interpolate_funct": interpolate_funct})
    _close(img, z[f"{k}_interp_img"])
    _close(mean_t[:, steps], z[f"{k}_interp_mean_t"])
    t = int(z["pmv_t"])
    for c in ("clip", "noclip"):
        mean, var, lv, x0 = d.p_mean_variance(start, torch.full((4,), t, device=cuda), clip_denoised=(c == "clip"))
        _close(x0, z[f"{k}_pmv_{c}_x0"])
        _close(mean, z[f"{k}_pmv_{c}_mean"])
        _close(var, z[f"{k}_pmv_{c}_var"])
        _close(lv, z[f"{k}_pmv_{c}_logvar"])
    for graph in (False, True):
        d.engine.enable_graph(graph)
        img, (_, _, mean_t) = d.sample(batch_size=4, start_noise=start, sampling_noise=samp, return_sampling_noise=True,
                                       clip_denoised=False)
        _close(img, z[f"{k}_noclip_img"])
        _close(mean_t[:, steps], z[f"{k}_noclip_mean_t"])


def test_release_no_clip(cuda):
    """clip_denoised=False on the nonisotropic release sampler (x0 pushed past +-1): the update
    kernel's clamp is off under SD_FLAG_NO_CLIP; sample (eager + hipGraph, 1 and 3 row chains),
    the interpolation path and one p_sample step against the reference."""
    z = golden("noclip_h36m16_T10")
    d = build_release_diffusion(z, cuda)
    xc, start, samp, noise2 = (t.to(cuda) for t in variant_inputs(z))
    B = start.shape[0]
    for graph in (False, True):
        d.engine.enable_graph(graph)
        img, (_, _, mean_t) = d.sample(batch_size=B, x_cond=xc, start_noise=start, sampling_noise=samp,
                                       return_sampling_noise=True, clip_denoised=False)
        _close(img, z["img"])
        _close(mean_t, z["mean_t"])
        clipped = d.sample(batch_size=B, x_cond=xc, start_noise=start, sampling_noise=samp)[0]
        assert float(clipped.abs().max()) <= 1.0 + 1e-6 < float(img.abs().max())
    img, _ = d.sample(batch_size=B, x_cond=xc, start_noise=start, sampling_noise=samp, if_interpolate=True,
                      noise2interpolate=noise2, interpolation_kwargs={"interpolate_funct": interpolate_funct},
                      clip_denoised=False)
    _close(img, z["interp_img"])
    t = int(z["step_t"])
    x, x0, noise, mean = d.p_sample(start, t, None, clip_denoised=False, sampling_noise=samp, x_cond=xc)
    _close(x0, z["step_x0"])
    _close(mean, z["step_mean"])
    _close(x, z["step_x"])


def test_no_clip_row_chains_and_device_noise(cuda):
    """SD_FLAG_NO_CLIP with device noise on three row chains equals one chain bitwise, and differs
    from the clamped chain (the flag reaches every chain's update)."""
    z = golden("noclip_h36m16_T10")
    d = build_release_diffusion(z, cuda)
    xc = torch.rand((4, 16, 96), generator=torch.Generator().manual_seed(5)).to(cuda) * 2 - 1
    res = {}
    for n in (1, 3):
        d.engine.set_option("row_chains", n)
        res[n] = d.engine.sample_loop(96, x_cond=xc, seed=3, graph=True, clip=False)[0].clone()
        assert d.engine.get_option("last_chains") == n
    clipped = d.engine.sample_loop(96, x_cond=xc, seed=3, graph=True)[0]
    torch.cuda.synchronize()
    assert torch.equal(res[1], res[3])
    assert not torch.equal(res[1], clipped)


@pytest.mark.parametrize("name", list(OPTION_CASES))
@pytest.mark.parametrize("model", ["readme", "release"])
def test_diffusion_options_match_reference(name, model, cuda):
    """the reference's config-selectable options sampled on the engine against
    the reference's own chains (every posterior table comes from the module's buffers; exp runs
    T + 1 = 11 steps)."""
    from conftest import option_inputs

    z = golden(f"option_{name}")
    d = build_option_diffusion(name, model, z, cuda)
    assert d.num_timesteps == int(z["num_timesteps"])
    _, _, xc, start, samp = option_inputs(z, model)
    kw = {} if xc is None else {"x_cond": xc.to(cuda)}
    img, (_, _, mean_t) = d.sample(batch_size=start.shape[0], start_noise=start.to(cuda),
                                   sampling_noise=samp.to(cuda), return_sampling_noise=True, **kw)
    _close(img, z[f"{model}_img"])
    _close(mean_t[:, z["mean_t_steps"]], z[f"{model}_mean_t"])
