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
    L = _lib.lib()
    res = {}
    try:
        for v in (0, 1):
            L.sd_set_update_kernel(v)
            a = eng.sample_loop(rows, x_cond=x_cond, seed=4, sampling_noise=samp, record=(True, False), graph=False)
            b = eng.sample_loop(rows, x_cond=x_cond, seed=4, sampling_noise=samp, record=(False, True), graph=False)
            torch.cuda.synchronize()
            res[v] = [t.clone() for t in (a[0], a[1], a[2], a[3], b[4])]  # img, start, noise_t, mean_t, imgs
    finally:
        L.sd_set_update_kernel(1)
    for name, x, y in zip(("img", "start", "noise_t", "mean_t", "imgs"), res[0], res[1]):
        assert torch.equal(x, y), (name, float((x - y).abs().max()))
    assert L.sd_set_update_kernel(-1) == 1 and L.sd_set_update_kernel(2) < 0
