"""GPU: the posterior update on the matrix cores (k_update_mfma, sd_kernels.hip) against the
element-per-thread forms (k_update / k_update_row) it replaces, bitwise -- latents, posterior
means, noise and timages records -- over the row counts of both of its workgroup shapes (one row
and four rows per workgroup), J = 16 / 17 / 21 and the J <= 64 form (MANO J = 51 / 52), device and given noise, f32 and bf16 latents
(reference op: nonisotropic.py:196-210 q_posterior + p_sample; the oracle parity of the whole
chain is in test_gpu_parity.py / test_gpu_configs.py)."""
import pytest
import torch

from skeletondiffusion_amd import _lib

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg,batch,prec", [("amass16", 64, "f32"), ("amass16", 1, "f32"), ("amass16", 21, "f32"),
                                            ("freeman17", 8, "f32"), ("amass21", 30, "f32"), ("freeman17", 24, "bf16"),
                                            ("mano51", 2, "f32"), ("mano52", 1, "f32")])
@pytest.mark.parametrize("given", [False, True])
def test_update_mfma_bitwise_vs_elementwise(cfg, batch, prec, given, cuda):
    from bench import build_config

    d, x_cond, rows = build_config(cfg, cuda, T=10, batch=batch)
    eng = d.engine
    eng.set_precision(prec)
    J = d.channels
    g = torch.Generator().manual_seed(11)
    samp = torch.randn((rows, 9, J, 96), generator=g).to(cuda) if given else None
    res = {}
    # SD_OPT_UPDATE_KERNEL: 1 the element-per-thread forms, 0 (default) k_update_mfma
    for v in (1, 0):
        eng.set_option("update_kernel", v)
        a = eng.sample_loop(rows, x_cond=x_cond, seed=4, sampling_noise=samp, record=(True, False), graph=False)
        b = eng.sample_loop(rows, x_cond=x_cond, seed=4, sampling_noise=samp, record=(False, True), graph=False)
        torch.cuda.synchronize()
        res[v] = [t.clone() for t in (a[0], a[1], a[2], a[3], b[4])]  # img, start, noise_t, mean_t, imgs
    for name, x, y in zip(("img", "start", "noise_t", "mean_t", "imgs"), res[0], res[1]):
        assert torch.equal(x, y), (name, float((x - y).abs().max()))
    assert eng.get_option("update_kernel") == 0
    for bad in (2, 3, 4):  # 2 / 3: the measured-no-faster forms ABI 3 removed
        with pytest.raises(_lib.SkelDiffError):
            eng.set_option("update_kernel", bad)


@pytest.mark.parametrize("dim,batch", [(192, 5), (192, 40), (160, 3), (256, 2)])
def test_update_mfma_wide_latents(dim, batch, cuda):
    """Latent widths beyond the 96 of the release configs (check_dims admits any multiple of 16):
    the matrix-core update covers at most 8 column tiles per row at one row per workgroup and 6 at
    four, so D = 160 / 192 / 256 must take a form that writes every column (advisor finding, round
    3) -- bitwise equal to the element-per-thread forms, with every column finite and written."""
    from conftest import pinned_cov
    from skeletondiffusion_amd import synthetic
    from skeletondiffusion_amd.core.diffusion import NonisotropicGaussianDiffusion
    from skeletondiffusion_amd.core.network import Denoiser

    J, T = 16, 4
    m = Denoiser(dim=dim, cond_dim=0, out_dim=dim, channels=J, num_nodes=J, depth=1, attn_heads=2,
                 attn_dim_head=32, learn_influence=True)
    synthetic.fill_module_(m, 77)
    S, L, U = pinned_cov(J)
    d = NonisotropicGaussianDiffusion(Sigma_N=S, Lambda_N=L, U=U, model=m, latent_size=dim, diffusion_timesteps=T,
                                      diffusion_objective="pred_x0", beta_schedule="cosine").to(cuda).eval()
    eng = d.engine
    rows = batch * 3
    res = {}
    for v in (1, 0):
        eng.set_option("update_kernel", v)
        sentinel = torch.full((rows, J, dim), float("nan"), device=cuda)
        a = eng.sample_loop(rows, seed=9, record=(True, False), graph=False, out=sentinel)
        torch.cuda.synchronize()
        res[v] = [t.clone() for t in (a[0], a[2], a[3])]  # img, noise_t, mean_t
        assert torch.isfinite(res[v][0]).all() and torch.isfinite(res[v][2]).all(), v
    for name, x, y in zip(("img", "noise_t", "mean_t"), res[0], res[1]):
        assert torch.equal(x, y), (name, float((x - y).abs().max()))
