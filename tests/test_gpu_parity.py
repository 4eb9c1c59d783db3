"""GPU parity: the HIP sampling engine (libskeldiff.so, called through the C ABI) against the
reference's own outputs (tests/golden) and against the CPU oracle on identical inputs.

Tolerance: generated latents within 1e-4 absolute (fp32; BASELINE.json north_star).  The
reference's own fp32-vs-fp64 drift is <= 1.1e-7, so the bar has headroom."""
import ctypes

import numpy as np
import pytest
import torch

import oracle as O
from conftest import (RELEASE_FIXTURES, WEIGHT_SEED, build_readme_diffusion, build_release_diffusion, golden,
                      pinned_cov, release_inputs)
from skeletondiffusion_amd import _lib

pytestmark = pytest.mark.gpu
TOL = 1e-4


def _max_err(a, b):
    a = a.detach().float().cpu().numpy() if torch.is_tensor(a) else np.asarray(a)
    b = b.detach().float().cpu().numpy() if torch.is_tensor(b) else np.asarray(b)
    return float(np.abs(a - b).max()) if a.size else 0.0


@pytest.mark.config_parity
@pytest.mark.parametrize("name", RELEASE_FIXTURES)
def test_release_sample_matches_reference(name, cuda):
    z = golden(name)
    d = build_release_diffusion(z, cuda)
    xcs, fu, start, samp = release_inputs(z)
    B = start.shape[0]
    img, (noise0, noise_t, mean_t) = d.sample(batch_size=B, x_cond=xcs.to(cuda), start_noise=start.to(cuda),
                                               sampling_noise=samp.to(cuda), return_sampling_noise=True)
    assert img.shape == (B, z["corr"].shape[0], 96)
    assert _max_err(img, z["img"]) < TOL
    m = mean_t.cpu()
    if "mean_t_steps" in z:
        m = m[:, z["mean_t_steps"]]
    assert _max_err(m, z["mean_t"]) < TOL
    assert _max_err(noise0, start) == 0.0 and _max_err(noise_t, samp) == 0.0


@pytest.mark.parametrize("variant", [3, 2, 1])
@pytest.mark.parametrize("name", ["release_h36m16_T10", "release_freeman17_T10"])
def test_exact_f32_generations_match_reference(name, variant, cuda):
    """The exact-f32 graph-linear generations (row-major activations, separate k_attention) on
    the whole sampler, against the same reference outputs as the default split-f16 v4 path."""
    z = golden(name)
    d = build_release_diffusion(z, cuda)
    d.engine.set_option("kernel_variant", variant)
    xcs, fu, start, samp = release_inputs(z)
    img, _ = d.sample(batch_size=start.shape[0], x_cond=xcs.to(cuda), start_noise=start.to(cuda),
                      sampling_noise=samp.to(cuda))
    assert _max_err(img, z["img"]) < TOL
    assert d.engine.get_option("kernel_variant") == variant


@pytest.mark.parametrize("name", ["release_h36m16_T10", "release_amass21_T10"])
def test_denoiser_forward_and_activations(name, cuda):
    z = golden(name)
    d = build_release_diffusion(z, cuda)
    xcs, fu, start, _ = release_inputs(z)
    x0 = d.engine.denoiser_forward(start.to(cuda), int(z["T"]) - 1, xcs.to(cuda))
    assert _max_err(x0, z["fwd_x0"]) < 1e-5


@pytest.mark.config_parity
@pytest.mark.parametrize("mode", ["noniso", "iso_as_noniso", "isotropic"])
def test_readme_config_matches_reference(mode, cuda):
    """BASELINE config 1: README plug-and-play Denoiser (no node types, G = I buffer)."""
    from skeletondiffusion_amd import synthetic

    z = golden("readme16_T10")
    d = build_readme_diffusion(mode, cuda)
    start = torch.from_numpy(synthetic.normal((4, 16, 96), 11)).to(cuda)
    samp = torch.from_numpy(synthetic.normal((4, 9, 16, 96), 12)).to(cuda)
    img, (_, _, mean_t) = d.sample(batch_size=4, start_noise=start, sampling_noise=samp, return_sampling_noise=True)
    assert _max_err(img, z[f"{mode}_img"]) < TOL
    assert _max_err(mean_t, z[f"{mode}_mean_t"]) < TOL


@pytest.mark.parametrize("obj", ["pred_noise", "pred_v"])
@pytest.mark.parametrize("act", ["identity", "tanh"])
def test_isotropic_objectives_match_reference(obj, act, cuda):
    """IsotropicGaussianDiffusion sampled with the pred_noise / pred_v objectives (isotropic.py:48-70,
    base.py:219-241): the update kernel forms x0 = a[t] x_t - b[t] act(model_out) before the clamp;
    sample() and p_sample() against the reference's own outputs (tests/golden/iso_objectives_T10.npz)."""
    from skeletondiffusion_amd import synthetic
    from skeletondiffusion_amd.core.diffusion import IsotropicGaussianDiffusion
    from skeletondiffusion_amd.core.network import Denoiser

    z = golden("iso_objectives_T10")
    m = Denoiser(dim=96, cond_dim=0, out_dim=96, channels=16, num_nodes=16)
    synthetic.fill_module_(m, WEIGHT_SEED)
    d = IsotropicGaussianDiffusion(model=m, diffusion_timesteps=10, diffusion_objective=obj,
                                   diffusion_activation=act).to(cuda).eval()
    start = torch.from_numpy(z["start"]).to(cuda)
    samp = torch.from_numpy(z["samp"]).to(cuda)
    img, (_, _, mean_t) = d.sample(batch_size=4, start_noise=start, sampling_noise=samp, return_sampling_noise=True)
    assert _max_err(img, z[f"{obj}_{act}_img"]) < TOL
    assert _max_err(mean_t, z[f"{obj}_{act}_mean_t"]) < TOL
    # one p_sample step (its x_start return is the predicted start, clamped)
    x, x_start, _, mean = d.p_sample(start, 9, sampling_noise=samp)
    assert _max_err(mean, z[f"{obj}_{act}_mean_t"][:, 0]) < TOL
    assert float(x_start.abs().max()) <= 1.0


def test_nonisotropic_objective_refusal_text(cuda):
    """The nonisotropic sampler takes pred_x0 only (the release configs; the reference's pred_v is
    'Not implemented', nonisotropic.py:122-124): the engine refuses others with a pinned message."""
    from skeletondiffusion_amd._lib import SkelDiffError

    d = build_readme_diffusion("noniso", cuda)
    d.objective = "pred_noise"
    with pytest.raises(SkelDiffError, match="objective 'pred_noise' on the nonisotropic sampler"):
        d.sample(batch_size=2)


def test_philox_device_stream_bit_exact(cuda):
    L = _lib.lib()
    rows, quads, seed, row0, step = 37, 24, 0x123456789ABCDEF, 1 << 33, 7
    out = torch.empty(rows * quads * 4, dtype=torch.int32, device=cuda)
    _lib.check(L.sd_philox_raw(out.data_ptr(), rows, quads, seed, row0, step, torch.cuda.current_stream().cuda_stream))
    got = out.cpu().numpy().view(np.uint32).reshape(rows, quads, 4)
    r = np.arange(row0, row0 + rows, dtype=np.uint64)[:, None]
    q = np.broadcast_to(np.arange(quads, dtype=np.uint32)[None], (rows, quads))
    exp = O.philox4x32_10(q, np.full_like(q, step), (r & 0xFFFFFFFF).astype(np.uint32) + 0 * q,
                          (r >> 32).astype(np.uint32) + 0 * q, seed & 0xFFFFFFFF, seed >> 32)
    for k in range(4):
        np.testing.assert_array_equal(got[..., k], exp[k])
    # the published KAT through the device path: ctr (0,0,0,0), key (0,0)
    kat = torch.empty(4, dtype=torch.int32, device=cuda)
    _lib.check(L.sd_philox_raw(kat.data_ptr(), 1, 1, 0, 0, 0, 0))
    torch.cuda.synchronize()
    assert tuple(kat.cpu().numpy().view(np.uint32)) == (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)


def test_device_normals_match_oracle(cuda):
    """Device Box-Muller (hardware log2 / sqrt / sin / cos) against the oracle's float64 transform
    of the same Philox words, over one config-2 step's 4.9 M normals (tails to |z| ~ 5.9)."""
    rows, n, seed, row0, step = 3200, 16 * 96, 99, 5, 3
    out = torch.empty((rows, n), device=cuda)
    _lib.check(_lib.lib().sd_noise_fill(out.data_ptr(), rows, n, seed, row0, step, 0))
    torch.cuda.synchronize()
    exp = O.philox_normal(seed, np.arange(row0, row0 + rows), step, n)
    err = _max_err(out, exp)
    assert err < 2e-5, err
    got = out.cpu().double()
    assert abs(float(got.mean())) < 5e-3 and abs(float(got.std()) - 1.0) < 5e-3


def test_device_noise_chain_matches_oracle(cuda):
    """Throughput mode (noise drawn on device) against the oracle fed the same Philox normals."""
    z = golden("release_h36m16_T10")
    d = build_release_diffusion(z, cuda)
    xcs, fu, _, _ = release_inputs(z)
    B, J, T, seed = 8, 16, 10, 4242
    img, (start, noise_t, _) = d.sample(batch_size=B, x_cond=xcs.to(cuda), seed=seed, return_sampling_noise=True)
    st, sn = O.device_noise(seed, 0, B, T, J, 96)
    assert _max_err(start, st) < 2e-5 and _max_err(noise_t, sn) < 2e-5
    cfg = O.release_config(J, z["node_types"])
    sd = O.synthetic_state_dict(cfg, WEIGHT_SEED)
    S, L, U = pinned_cov(J)
    bufs = O.nonisotropic_buffers(S, L, U, O.beta_schedule("cosine", T))
    ref, _ = O.p_sample_loop(sd, cfg, bufs, st, sn, x_cond=xcs)
    assert _max_err(img, ref) < TOL


def test_graph_replay_equals_eager_bitwise(cuda):
    z = golden("release_h36m16_T10")
    d = build_release_diffusion(z, cuda)
    xc = release_inputs(z)[0].to(cuda)
    a = d.engine.sample_loop(8, x_cond=xc, seed=77, graph=False)[0]
    out = torch.empty_like(a)
    # `out` is reused so the captured graph is replayed: clone each result before the next call
    b = d.engine.sample_loop(8, x_cond=xc, seed=77, graph=True, out=out, keep_start=False)[0].clone()
    c = d.engine.sample_loop(8, x_cond=xc, seed=77, graph=True, out=out, keep_start=False)[0].clone()
    e = d.engine.sample_loop(8, x_cond=xc, seed=78, graph=True, out=out, keep_start=False)[0].clone()
    torch.cuda.synchronize()
    assert torch.equal(a, b) and torch.equal(a, c)
    assert not torch.equal(a, e)


def test_row0_makes_noise_shard_invariant(cuda):
    """Rows split across launches (or GPUs) with the right row0 give bitwise the same latents."""
    z = golden("release_h36m16_T10")
    d = build_release_diffusion(z, cuda)
    xcs = release_inputs(z)[0].to(cuda)                 # 2 sequences x 4 futures
    full = d.sample(batch_size=8, x_cond=xcs, seed=5)[0]
    lo = d.sample(batch_size=4, x_cond=xcs[:1], seed=5, row0=0)[0]
    hi = d.sample(batch_size=4, x_cond=xcs[1:], seed=5, row0=4)[0]
    assert torch.equal(full, torch.cat([lo, hi]))


@pytest.mark.parametrize("B", [1, 3, 67])
def test_ragged_batches(B, cuda):
    """Batch sizes that do not fill a 64-row tile; x_cond given per row."""
    z = golden("release_freeman17_T10")
    d = build_release_diffusion(z, cuda)
    J = 17
    g = torch.Generator().manual_seed(B)
    xc = torch.rand((B, J, 96), generator=g) * 2 - 1
    start = torch.randn((B, J, 96), generator=g)
    samp = torch.randn((B, 9, J, 96), generator=g)
    img = d.sample(batch_size=B, x_cond=xc.to(cuda), start_noise=start.to(cuda), sampling_noise=samp.to(cuda))[0]
    cfg = O.release_config(J, z["node_types"])
    sd = O.synthetic_state_dict(cfg, WEIGHT_SEED)
    S, L, U = pinned_cov(J)
    bufs = O.nonisotropic_buffers(S, L, U, O.beta_schedule("cosine", 10))
    ref, _ = O.p_sample_loop(sd, cfg, bufs, start, samp, x_cond=xc)
    assert _max_err(img, ref) < TOL


def test_empty_batch(cuda):
    """rows == 0 is a no-op at the ABI level."""
    z = golden("release_h36m16_T10")
    d = build_release_diffusion(z, cuda)
    L = _lib.lib()
    plan = d.engine.plan()
    ws, nb = d.engine.workspace(1)
    rc = L.sd_sample_loop(plan, None, ws.data_ptr(), 1, None, 1, 0, ws.data_ptr(), None, None, None, None, 0,
                          ws.data_ptr(), nb, 6, 0)
    assert rc == 0


def test_single_step_p_sample(cuda):
    z = golden("release_amass21_T10")
    d = build_release_diffusion(z, cuda)
    xcs, fu, start, samp = release_inputs(z)
    t = 5
    eps = samp[:, 9 - t]
    img, x0, noise, mean = d.p_sample(start.to(cuda), t, None, sampling_noise=samp.to(cuda), x_cond=xcs.to(cuda))
    J = 21
    cfg = O.release_config(J, z["node_types"])
    sd = O.synthetic_state_dict(cfg, WEIGHT_SEED, float(z["final_scale"]))
    S, L, U = pinned_cov(J)
    bufs = O.nonisotropic_buffers(S, L, U, O.beta_schedule("cosine", 10))
    xc = xcs.repeat_interleave(fu, 0)
    out = O.denoiser_forward(sd, cfg, start, torch.full((4,), t), xc).clamp(-1, 1)
    m = bufs["posterior_mean_coef1_x0"][t] @ out + bufs["posterior_mean_coef2_xt"][t] @ start
    ref = m + bufs["U"] @ ((0.5 * bufs["Lambda_posterior_log_variance_clipped"][t]).exp()[:, None] * eps)
    assert _max_err(x0, out) < 1e-5 and _max_err(mean, m) < 1e-5 and _max_err(img, ref) < 1e-5
    assert _max_err(noise, eps) == 0.0


def test_weights_update_rebuilds_plan(cuda):
    z = golden("release_h36m16_T10")
    d = build_release_diffusion(z, cuda)
    xcs, fu, start, samp = release_inputs(z)
    a = d.engine.denoiser_forward(start.to(cuda), 3, xcs.to(cuda))
    with torch.no_grad():
        d.model.final_glin.bias.add_(1.0)
    b = d.engine.denoiser_forward(start.to(cuda), 3, xcs.to(cuda))
    assert _max_err(a, b) > 0.1


def test_full_size_config2_step_and_properties(cuda):
    """BASELINE config 2 at full size: J=16, B=64x50=3200, T=100, release architecture.
    One denoiser step against the oracle at full size, then size-independent properties of the
    whole chain: finite, deterministic, shard invariant, t=0 output = clamp(x0) in [-1, 1]."""
    from bench import build_config

    d, x_cond, rows = build_config("amass16", cuda, T=100)
    x = torch.randn((rows, 16, 96), generator=torch.Generator().manual_seed(0))
    t = 63
    got = d.engine.denoiser_forward(x.to(cuda), t, x_cond)
    cfg = O.release_config(16, d.model.node_types)
    sd = {k: v.detach().cpu() for k, v in d.state_dict().items()}
    ref = O.denoiser_forward(sd, cfg, x, torch.full((rows,), t), x_cond.cpu().repeat_interleave(rows // x_cond.shape[0], 0))
    assert _max_err(got, ref) < TOL
    a = d.sample(batch_size=rows, x_cond=x_cond, seed=11)[0]
    b = d.sample(batch_size=rows, x_cond=x_cond, seed=11)[0]
    assert torch.isfinite(a).all() and torch.equal(a, b)
    assert a.abs().max() <= 1.0 + 1e-5  # t = 0: C1[0] = I, C2[0] = 0, no noise -> clamp(x0)
    part = d.sample(batch_size=100, x_cond=x_cond[6:8], seed=11, row0=300)[0]
    assert torch.equal(part, a[300:400])


@pytest.mark.parametrize("route", [1, 0])
@pytest.mark.parametrize("graph", [False, True])
def test_row_chains_bitwise_invariant(graph, route, cuda):
    """SD_OPT_ROW_CHAINS: the batch is split into row ranges whose T-step chains run on forked
    streams.  Rows are independent, so latents and every per-step record are bitwise those of a
    single chain -- device noise (row0-shifted Philox) and given noise (row-offset eps) alike --
    on the one-kernel route (split_route 1) and the auto route (k_gl4y at this size); the chain
    count each call ran is asserted (SD_OPT_LAST_CHAINS)."""
    z = golden("release_h36m16_T10")
    d = build_release_diffusion(z, cuda)
    J, T = 16, 10
    g = torch.Generator().manual_seed(3)
    # 17 sequences x 6 futures = 102 rows: 3 chain units of 32 rows + a ragged 6-row unit (up to 4
    # chains, the last one 6 rows); chains start inside a sequence's futures (row 32 = sequence 5,
    # future 2), exercising the x_cond phase
    xc = (torch.rand((17, J, 96), generator=g) * 2 - 1).to(cuda)
    rows = 102
    start = torch.randn((rows, J, 96), generator=g).to(cuda)
    samp = torch.randn((rows, T - 1, J, 96), generator=g).to(cuda)
    L = _lib.lib()
    d.engine.set_option("split_route", route)
    res = {}
    for n in (1, 2, 3, 8):
        d.engine.set_option("row_chains", n)
        a = d.engine.sample_loop(rows, x_cond=xc, seed=21, row0=7, record=(True, False), graph=graph)
        b = d.engine.sample_loop(rows, x_cond=xc, start_noise=start, sampling_noise=samp, record=(False, True),
                                 graph=graph)
        torch.cuda.synchronize()
        assert d.engine.get_option("last_chains") == min(n, (rows + 31) // 32)
        res[n] = [t.clone() for t in (a[0], a[1], a[2], a[3], b[0], b[4])]
    for n in (2, 3, 8):
        for x, y in zip(res[1], res[n]):
            assert torch.equal(x, y), n
    with pytest.raises(_lib.SkelDiffError):
        d.engine.set_option("row_chains", 9)
    with pytest.raises(_lib.SkelDiffError):
        d.engine.set_option("last_chains", 1)


def test_sharded_eval_single_rank(cuda):
    """skeletondiffusion_amd.sharded on one rank: the shard is the whole batch, row0 = 0, and the
    metric reduction is the plain mean (the world > 1 paths run under gloo in test_distributed)."""
    from skeletondiffusion_amd import metrics, sharded

    z = golden("release_h36m16_T10")
    d = build_release_diffusion(z, cuda)
    xcs = release_inputs(z)[0].to(cuda)
    out, s0 = sharded.sample_sharded(lambda **kw: d.sample(**kw)[0], xcs, 4, seed=9)
    ref = d.sample(batch_size=8, x_cond=xcs, seed=9, row0=0)[0]
    assert s0 == 0 and torch.equal(out, ref)
    v = metrics.lat_apd(out.view(2, 4, 16, 96))
    assert abs(sharded.reduce_metric(v, nseq_total=2).item() - v.double().mean().item()) < 1e-6
