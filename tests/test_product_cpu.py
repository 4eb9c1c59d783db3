"""Host-side product logic on CPU: the reference API surface (constructors, attributes,
state_dict, buffers, training forward) against the reference's own outputs, and the
no-CPU-sampling rule."""
import re
import numpy as np
import pytest
import torch

from conftest import RELEASE_FIXTURES, build_readme_diffusion, build_release_diffusion, golden, release_inputs
from skeletondiffusion_amd import synthetic
from skeletondiffusion_amd._lib import SkelDiffError


@pytest.mark.parametrize("name", ["release_h36m16_T10", "release_amass21_T10"])
def test_release_module_forward_and_loss(name):
    z = golden(name)
    d = build_release_diffusion(z)
    xcs, fu, start, _ = release_inputs(z)
    xc = xcs.repeat_interleave(fu, 0)
    B, T = start.shape[0], int(z["T"])
    with torch.no_grad():
        x0 = d.model(start, torch.full((B,), T - 1), None, xc)
    np.testing.assert_allclose(x0.numpy(), z["fwd_x0"], atol=1e-6, rtol=0)
    J = start.shape[1]
    t_train = torch.arange(B) % T
    noise = torch.from_numpy(synthetic.normal((B, J, 96), 24))
    xs = torch.from_numpy(synthetic.uniform((B, J, 96), 25))
    loss, lw, mout = d.p_losses(xs, t_train, noise=noise, x_cond=xc)
    np.testing.assert_allclose(loss.detach().numpy(), z["train_loss"], atol=1e-6, rtol=1e-6)
    np.testing.assert_array_equal(lw.numpy(), z["train_loss_weight"])
    np.testing.assert_allclose(mout.detach().numpy(), z["train_model_out"], atol=1e-6, rtol=0)
    loss.mean().backward()  # forward() stays autograd-capable
    assert d.model.init_lin.G.grad is not None and torch.isfinite(d.model.init_lin.weight.grad).all()


@pytest.mark.parametrize("key", ["h36m16", "amass21", "mano51", "freeman17", "mano52"])
def test_buffers_bit_exact(key):
    from skeletondiffusion_amd.core.diffusion import NonisotropicGaussianDiffusion, get_cov_from_corr
    from skeletondiffusion_amd.core.network import Denoiser

    z = golden("cov_" + key)
    J = z["corr"].shape[0]
    S, L, U = get_cov_from_corr(torch.from_numpy(z["corr"]))
    for T in (10, 100):
        d = NonisotropicGaussianDiffusion(Sigma_N=S, Lambda_N=L, U=U, diffusion_timesteps=T,
                                          model=Denoiser(dim=96, out_dim=96, channels=J, num_nodes=J))
        for k, v in d.state_dict().items():
            if k.startswith("model."):
                continue
            v = v.numpy()
            if v.ndim == 3 and T == 100:
                v = v[[0, 1, 50, 99]]
            np.testing.assert_array_equal(v, z[f"T{T}_buf_{k}"], err_msg=f"{key} {k}")


@pytest.mark.parametrize("mode", ["noniso", "iso_as_noniso", "isotropic"])
def test_readme_modules(mode):
    z = golden("readme16_T10")
    d = build_readme_diffusion(mode)
    for k, v in d.state_dict().items():
        if not k.startswith("model."):
            np.testing.assert_array_equal(v.numpy(), z[f"{mode}_buf_{k}"], err_msg=k)
    assert d.num_timesteps == 10 and d.objective == "pred_x0" and d.channels == 16
    x = torch.from_numpy(synthetic.uniform((8, 16, 96), 13, 0.0, 1.0))
    noise = torch.from_numpy(synthetic.normal((8, 16, 96), 14))
    loss, lw, mout = d.p_losses(x, torch.from_numpy(z["train_t"]), noise=noise)
    np.testing.assert_allclose(loss.detach().numpy(), z[f"{mode}_loss"], atol=1e-6, rtol=1e-6)
    np.testing.assert_allclose(mout.detach().numpy(), z[f"{mode}_model_out"], atol=1e-6, rtol=0)


def test_state_dict_strict_roundtrip():
    """A state_dict from one module loads strictly into another (the eval.py checkpoint path,
    reference src/eval_prepare_model.py:69-72)."""
    z = golden("release_h36m16_T10")
    a = build_release_diffusion(z)
    b = build_release_diffusion(z)
    with torch.no_grad():
        for p in b.parameters():
            p.zero_()
    b.load_state_dict(a.state_dict(), strict=True)
    assert len(a.state_dict()) == 137
    for (ka, va), (kb, vb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert ka == kb and torch.equal(va, vb)


def test_sample_on_cpu_raises():
    d = build_readme_diffusion("noniso")
    with pytest.raises(SkelDiffError, match="HIP engine"):
        d.sample(batch_size=2)


@pytest.mark.parametrize("kw, reason", [
    (dict(self_condition=True), "self_condition"),
    (dict(learned_variance=True), "learned_variance"),
    (dict(learned_sinusoidal_cond=True), "learned/random sinusoidal time embedding"),
    (dict(random_fourier_features=True), "learned/random sinusoidal time embedding"),
])
def test_non_release_denoiser_options_refused_with_reason(kw, reason):
    """Denoiser options no release config uses (generator.py:16-45,80,88) build as torch modules
    like the reference's, and the sampling engine refuses them by name at plan time instead of
    sampling something else (engine.py:_desc).  norm_type='layer' (attention.py:55-60) runs on the
    engine since round 6 (tests/test_gpu_layernorm.py)."""
    from skeletondiffusion_amd.core.diffusion import NonisotropicGaussianDiffusion, get_cov_from_corr
    from skeletondiffusion_amd.core.network import Denoiser

    m = Denoiser(dim=96, cond_dim=0, out_dim=96, channels=16, num_nodes=16, **kw)
    S, L, U = get_cov_from_corr(torch.eye(16))
    d = NonisotropicGaussianDiffusion(Sigma_N=S, Lambda_N=L, U=U, model=m, diffusion_timesteps=10)
    with pytest.raises(SkelDiffError, match="sampling engine does not support: " + re.escape(reason)):
        d.engine._desc()


def test_unknown_kwargs_are_swallowed():
    """Constructors swallow unknown kwargs like the reference."""
    from skeletondiffusion_amd.core.diffusion import NonisotropicGaussianDiffusion, get_cov_from_corr
    from skeletondiffusion_amd.core.network import Denoiser

    m = Denoiser(dim=96, cond_dim=0, out_dim=96, channels=16, num_nodes=16, arch="Denoiser", not_a_kwarg=3)
    S, L, U = get_cov_from_corr(torch.eye(16), foo=1)
    d = NonisotropicGaussianDiffusion(Sigma_N=S, Lambda_N=L, U=U, model=m, timesteps=10, whatever=3)
    assert d.num_timesteps == 10  # 'timesteps' is swallowed; diffusion_timesteps default applies


def test_ddim_is_rejected_like_reference():
    from skeletondiffusion_amd.core.diffusion import IsotropicGaussianDiffusion
    from skeletondiffusion_amd.core.network import Denoiser

    d = IsotropicGaussianDiffusion(model=Denoiser(dim=96, out_dim=96, channels=4, num_nodes=4),
                                   diffusion_timesteps=10, sampling_timesteps=5)
    assert d.is_ddim_sampling
    with pytest.raises(NotImplementedError):
        d.sample(batch_size=1)


def test_isotropic_covariance_type_fails_like_reference():
    from skeletondiffusion_amd.core.diffusion import NonisotropicGaussianDiffusion, get_cov_from_corr
    from skeletondiffusion_amd.core.network import Denoiser

    S, L, U = get_cov_from_corr(torch.eye(4), if_run_as_isotropic=True, diffusion_covariance_type="isotropic")
    with pytest.raises(RuntimeError):
        NonisotropicGaussianDiffusion(Sigma_N=S, Lambda_N=L, U=U, diffusion_covariance_type="isotropic",
                                      model=Denoiser(dim=96, out_dim=96, channels=4, num_nodes=4))


def test_hip_training_route_validates_shapes():
    """StaticGraphLinear routes to the HIP training kernels only for shapes they support (J <= 64,
    a (J, J) mixing matrix, node types indexing the weight): anything else stays on the torch
    path and fails with torch's own shape errors instead of out-of-bounds device reads."""
    from skeletondiffusion_amd.training import hip_shapes_ok

    x = torch.zeros(2, 16, 8)
    W3, W2 = torch.zeros(3, 4, 8), torch.zeros(4, 8)
    types = torch.tensor([0, 1, 2] * 5 + [0])
    assert hip_shapes_ok(x, W3, torch.eye(16), types)
    assert hip_shapes_ok(x, W2, torch.eye(16), None)
    assert not hip_shapes_ok(torch.zeros(2, 65, 8), W2, torch.eye(65), None)      # J > 64
    assert not hip_shapes_ok(x, W3, torch.eye(15), types)                           # ghat not (J, J)
    assert not hip_shapes_ok(x, W3, torch.eye(16), types[:15])                      # len(types) != J
    assert not hip_shapes_ok(x, W3, torch.eye(16), torch.full((16,), 3))            # type >= n_types
    assert not hip_shapes_ok(x, W3, torch.eye(16), None)                            # 3-D weight, no types
