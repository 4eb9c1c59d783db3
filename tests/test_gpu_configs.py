"""GPU parity on the BASELINE configurations as they are benched, and on the optional sample()
surface (VERDICT r01 "what's missing" 1-3):

* config 4 (Human3.6M J=16, one sequence x 50 futures, T=1000, hipGraph, device noise): the
  first 5 and the last 5 reverse steps against the oracle fed the same Philox normals, plus
  graph == eager bitwise, finiteness, determinism and the t = 0 clamp; the reference's own T=1000
  chain is in test_gpu_parity.py::test_release_sample_matches_reference[release_h36m16_T1000];
* config 2 exactly as bench.py times it (J=16, B=3200, T=100, 3 row chains on the tiled split
  route, hipGraph, reused output buffer, device noise): every per-step record bitwise equal to
  one chain run eagerly, and the first 3 steps against the oracle on the rows at the chain
  boundaries;
* row chains sharing CUs on every route and at the strong-scaling shard sizes,
  each asserting the chain count the call ran (SD_OPT_LAST_CHAINS);
* per-layer activations of the Denoiser (sd_denoiser_trace) against the reference's forward hooks;
* Denoiser(use_attention=False), diffusion_activation='tanh', return_timages and noise
  interpolation against the reference's outputs (tests/golden/variants_h36m16_T10.npz);
* two plans sampling concurrently in one process (different options; two default plans).

Tolerance: 1e-4 absolute on generated latents (north star); the per-layer activations 1e-5."""
import threading

import numpy as np
import pytest
import torch

import oracle as O
from conftest import (WEIGHT_SEED, build_release_diffusion, golden, interpolate_funct, release_inputs,
                      variant_inputs)
from skeletondiffusion_amd import _lib

pytestmark = pytest.mark.gpu
TOL = 1e-4


def _max_err(a, b):
    a = a.detach().float().cpu().numpy() if torch.is_tensor(a) else np.asarray(a)
    b = b.detach().float().cpu().numpy() if torch.is_tensor(b) else np.asarray(b)
    return float(np.abs(a - b).max()) if a.size else 0.0


def _oracle_setup(d):
    J = d.channels
    sd = {k: v.detach().cpu() for k, v in d.state_dict().items()}
    cfg = O.release_config(J, d.model.node_types)
    bufs = {k: v for k, v in sd.items() if not k.startswith("model.")}
    return sd, cfg, bufs


def _device_normals(seed, rows, step, J, D):
    return torch.from_numpy(O.philox_normal(seed, np.asarray(rows), step, J * D).reshape(len(rows), J, D))


@pytest.mark.config_parity
def test_config4_t1000_graph_first_and_last_steps(cuda):
    """BASELINE config 4: H36M J=16, 1 sequence x 50 futures, T=1000, hipGraph-captured chain."""
    from bench import build_config

    d, x_cond, rows = build_config("h36m_t1000", cuda)
    J, D, T = d.channels, d.seq_length, d.num_timesteps
    assert (rows, J, T) == (50, 16, 1000)
    seed, eng = 4711, d.engine
    out = torch.empty((rows, J, D), device=cuda)
    g = eng.sample_loop(rows, x_cond=x_cond, seed=seed, graph=True, out=out, record=(False, True))
    img_g, start, imgs = g[0].clone(), g[1].clone(), g[4]
    assert eng.get_option("last_chains") == 1  # auto: one chain at 128 rows and below
    g2 = eng.sample_loop(rows, x_cond=x_cond, seed=seed, graph=True, out=out, keep_start=False)[0].clone()
    e = eng.sample_loop(rows, x_cond=x_cond, seed=seed, graph=False)[0]
    eng.set_option("row_chains", 2)  # two chains of 32 + 18 rows (a ragged last 32-row unit)
    two = eng.sample_loop(rows, x_cond=x_cond, seed=seed, graph=True, record=(False, True))
    torch.cuda.synchronize()
    assert eng.get_option("last_chains") == 2
    eng.set_option("row_chains", 0)
    assert torch.isfinite(img_g).all() and img_g.abs().max() <= 1.0 + 1e-6  # t = 0: clamp(x0)
    assert torch.equal(img_g, g2) and torch.equal(img_g, e)
    assert torch.equal(img_g, two[0]) and torch.equal(imgs, two[4])  # chain-count invariant, every step
    sd, cfg, bufs = _oracle_setup(d)
    xc = x_cond.cpu()
    r = np.arange(rows)
    # first 5 steps from the device start noise (Philox step index T)
    st = _device_normals(seed, r, T, J, D)
    assert _max_err(start, st) < 2e-5
    x = st
    for k in range(5):
        t = T - 1 - k
        x, _ = O.p_sample_step(sd, cfg, bufs, x, t, _device_normals(seed, r, t, J, D), x_cond=xc)
        assert _max_err(imgs[:, k], x) < TOL, (k, _max_err(imgs[:, k], x))
    # last 5 steps (t = 4 .. 0) from the GPU's x_5 (the output of the step at t = 5)
    x = imgs[:, T - 1 - 5].cpu()
    for t in range(4, -1, -1):
        noise = _device_normals(seed, r, t, J, D) if t > 0 else 0.0
        x, _ = O.p_sample_step(sd, cfg, bufs, x, t, noise, x_cond=xc)
        ref = imgs[:, T - 1 - t] if t > 0 else img_g
        assert _max_err(ref, x) < TOL, (t, _max_err(ref, x))


@pytest.mark.config_parity
def test_config2_as_benched(cuda):
    """BASELINE config 2 with the bench's exact launch configuration: default plan options (the
    tiled split route, k_gl4t + k_gl4 MODE 2 / 3, on 3 row chains whose kernels share CUs),
    hipGraph, device noise, reused output buffer; every per-step record of the whole T = 100 chain
    bitwise equal to one chain run eagerly; first 3 steps vs the oracle on the rows either side of
    each chain boundary."""
    from bench import build_config

    d, x_cond, rows = build_config("amass16", cuda, T=100)
    J, D, T = d.channels, d.seq_length, d.num_timesteps
    eng, seed = d.engine, 20251015
    eng.set_option("row_chains", 3)
    out = torch.empty((rows, J, D), device=cuda)
    a = eng.sample_loop(rows, x_cond=x_cond, seed=seed, graph=True, out=out, record=(True, True))
    a = [t.clone() for t in (a[0], a[1], a[2], a[4])]  # img, start, noise_t, imgs
    assert eng.get_option("last_chains") == 3
    eng.set_option("row_chains", 1)
    b = eng.sample_loop(rows, x_cond=x_cond, seed=seed, graph=False, record=(True, True))
    b = [b[0], b[1], b[2], b[4]]
    assert eng.get_option("last_chains") == 1
    # the exact bench.py call (no records, output buffer reused, start not kept)
    eng.set_option("row_chains", 3)
    c = eng.sample_loop(rows, x_cond=x_cond, seed=seed, graph=True, out=out, keep_start=False)[0]
    assert eng.get_option("last_chains") == 3
    torch.cuda.synchronize()
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    assert torch.equal(c, a[0])
    img, start, imgs = a[0], a[1], a[3]
    assert torch.isfinite(img).all() and img.abs().max() <= 1.0 + 1e-6
    # the chain starts of a 3200-row, 3-chain split: rows 0, 1056, 2112 (multiples of 32)
    sel = np.concatenate([np.arange(0, 16), np.arange(1040, 1072), np.arange(2096, 2128), np.arange(3184, 3200)])
    sd, cfg, bufs = _oracle_setup(d)
    xc = x_cond.cpu().repeat_interleave(rows // x_cond.shape[0], 0)[sel]
    x = _device_normals(seed, sel, T, J, D)
    assert _max_err(start[sel], x) < 2e-5
    for k in range(3):
        t = T - 1 - k
        x, _ = O.p_sample_step(sd, cfg, bufs, x, t, _device_normals(seed, sel, t, J, D), x_cond=xc)
        assert _max_err(imgs[sel, k], x) < TOL, (k, _max_err(imgs[sel, k], x))


@pytest.mark.config_parity
def test_config3_as_benched(cuda):
    """BASELINE config 3's per-rank shard exactly as `bench.py --config mano51` times it (AMASS-MANO
    J = 51, 64 sequences x 50 futures = 3,200 rows, T = 100, default plan options: v5 with the
    split-f16 k_gl4t GEMM phase -- to_qkv on the 8-tile CT8 workgroups -- the k_gl5_mixd LDS-DMA
    mixing ring and k_attention, on 3 row chains sharing CUs, hipGraph, device noise, reused
    output buffer): every per-step record of the whole chain bitwise equal to one chain run
    eagerly; the first 3 steps against the oracle on the rows either side of each chain boundary."""
    from bench import build_config

    d, x_cond, rows = build_config("mano51", cuda, T=100)
    J, D, T = d.channels, d.seq_length, d.num_timesteps
    assert (rows, J, T) == (3200, 51, 100)
    eng, seed = d.engine, 20261018
    out = torch.empty((rows, J, D), device=cuda)
    a = eng.sample_loop(rows, x_cond=x_cond, seed=seed, graph=True, out=out, record=(True, True))
    a = [t.clone() for t in (a[0], a[1], a[2], a[4])]  # img, start, noise_t, imgs
    assert eng.get_option("last_chains") == 3  # auto at 3,200 rows
    bits = eng.get_option("last_route")
    assert bits & 8 and bits & 32 and bits & 128, bits  # k_gl4t GEMM phase, v5 mixing, k_attention
    eng.set_option("row_chains", 1)
    b = eng.sample_loop(rows, x_cond=x_cond, seed=seed, graph=False, record=(True, True))
    b = [b[0], b[1], b[2], b[4]]
    assert eng.get_option("last_chains") == 1
    eng.set_option("row_chains", 0)
    c = eng.sample_loop(rows, x_cond=x_cond, seed=seed, graph=True, out=out, keep_start=False)[0]
    assert eng.get_option("last_chains") == 3
    torch.cuda.synchronize()
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    assert torch.equal(c, a[0])
    img, start, imgs = a[0], a[1], a[3]
    assert torch.isfinite(img).all() and img.abs().max() <= 1.0 + 1e-6
    assert eng.status(rows) == 0
    # 3 chains of a 3,200-row call start at rows 0, 1056, 2112 (multiples of 32)
    sel = np.concatenate([np.arange(0, 8), np.arange(1048, 1064), np.arange(2104, 2120), np.arange(3192, 3200)])
    sd, cfg, bufs = _oracle_setup(d)
    xc = x_cond.cpu().repeat_interleave(rows // x_cond.shape[0], 0)[sel]
    x = _device_normals(seed, sel, T, J, D)
    assert _max_err(start[sel], x) < 2e-5
    for k in range(3):
        t = T - 1 - k
        x, _ = O.p_sample_step(sd, cfg, bufs, x, t, _device_normals(seed, sel, t, J, D), x_cond=xc)
        assert _max_err(imgs[sel, k], x) < TOL, (k, _max_err(imgs[sel, k], x))


@pytest.mark.parametrize("route,staging", [(1, 0), (1, 1), (3, 0), (2, 0)])
def test_row_chains_share_cus_bitwise(route, staging, cuda):
    """Row chains whose kernels share CUs (no whole-CU reservations) on each route
    -- one-kernel k_gl4 (LDS-DMA and register-staged weight stages), tiled k_gl4t + MODE 2 / 3,
    per-wave k_gl4y + MODE 2 / 3 -- at config 2's full batch (T = 10): 3 and 2 chains, graph and
    eager, bitwise equal to one chain; the chain count each call ran is asserted."""
    from bench import build_config

    d, x_cond, rows = build_config("amass16", cuda, T=10)
    eng = d.engine
    eng.set_option("split_route", route)
    eng.set_option("gl4_staging", staging)
    eng.set_option("row_chains", 1)
    ref = eng.sample_loop(rows, x_cond=x_cond, seed=3)[0].clone()
    assert eng.get_option("last_chains") == 1
    for n in (3, 2):
        eng.set_option("row_chains", n)
        for graph in (False, True):
            x = eng.sample_loop(rows, x_cond=x_cond, seed=3, graph=graph)[0]
            torch.cuda.synchronize()
            assert eng.get_option("last_chains") == n
            assert torch.equal(x, ref), (route, staging, n, graph, _max_err(x, ref))
    assert eng.status(rows) == 0


@pytest.mark.parametrize("batch", [32, 16, 8])
def test_strong_scaling_shards_chain_invariant(batch, cuda):
    """The per-rank shards of config 2 under strong scaling on 2 / 4 / 8 GPUs (1,600 / 800 / 400
    rows, J = 16 f32, T = 100, default routes): three row chains equal one chain bitwise over the
    whole T = 100 chain, graph replay and eager, with the chain count asserted."""
    from bench import build_config

    d, x_cond, rows = build_config("amass16", cuda, T=100, batch=batch)
    eng = d.engine
    eng.set_option("row_chains", 1)
    ref = eng.sample_loop(rows, x_cond=x_cond, seed=17, row0=rows)[0].clone()
    assert eng.get_option("last_chains") == 1
    eng.set_option("row_chains", 3)
    for graph in (True, False):
        x = eng.sample_loop(rows, x_cond=x_cond, seed=17, row0=rows, graph=graph)[0]
        torch.cuda.synchronize()
        assert eng.get_option("last_chains") == 3
        assert torch.equal(x, ref), (rows, graph, _max_err(x, ref))


@pytest.mark.parametrize("cfg,batch,kw", [("h36m_t1000", 1, {}), ("amass16", 4, {}), ("amass16", 12, {}),
                                          ("amass21", 4, {}), ("freeman17", 2, {}),
                                          ("amass16", 4, {"precision": "half"})])
def test_split_route_bitwise(cfg, batch, kw, cuda):
    """SD_OPT_SPLIT_ROUTE (DESIGN.md §4d'): the small-launch route 2 -- k_gl4y GEMM phase per
    (tile, node, column tile) + k_gl4 MODE 2 / 3 mixing or attention phase -- is bitwise equal to
    the one-kernel route, graph and eager, with the f16 range guard word untouched and the kernels
    the route launched asserted."""
    from bench import build_config

    d, x_cond, rows = build_config(cfg, cuda, T=10, batch=batch)
    eng = d.engine
    if kw.get("precision"):
        eng.set_precision(kw["precision"])
    eng.set_option("row_chains", 1)
    eng.set_option("split_route", 1)
    ref = eng.sample_loop(rows, x_cond=x_cond, seed=5, record=(False, True))
    ref = [ref[0].clone(), ref[4].clone()]
    eng.set_option("split_route", 2)
    for graph in (False, True):
        got = eng.sample_loop(rows, x_cond=x_cond, seed=5, graph=graph, record=(False, True))
        torch.cuda.synchronize()
        assert torch.equal(got[0], ref[0]) and torch.equal(got[4], ref[1]), (cfg, batch, graph)
    bits = eng.get_option("last_route")
    assert bits & 4 and bits & 16 and not bits & 3, bits  # k_gl4y + MODE 2 / 3, no one-kernel tile
    for bad in (5, 6):  # the measured-slower routes ABI 3 removed
        with pytest.raises(_lib.SkelDiffError):
            eng.set_option("split_route", bad)
    assert eng.status(rows) == 0


@pytest.mark.parametrize("cfg,batch,T,prec", [("amass16", 64, 4, "f32"), ("amass21", 8, 10, "f32"),
                                               ("freeman17", 8, 10, "f32"), ("freeman17", 16, 10, "half"),
                                               ("freeman17", 16, 10, "bf16"), ("amass21", 16, 10, "bf16")])
def test_tiled_split_route_bitwise(cfg, batch, T, prec, cuda):
    """SD_OPT_SPLIT_ROUTE = 3 (DESIGN.md §4d''): the tiled GEMM phase k_gl4t (128 rows x 192
    columns of one node per workgroup) + k_gl4 MODE 2 / 3 is bitwise equal to the one-kernel
    route, graph and eager, on one row chain and on three (sharing CUs, §4c)."""
    from bench import build_config

    d, x_cond, rows = build_config(cfg, cuda, T=T, batch=batch)
    eng = d.engine
    eng.set_precision(prec)
    eng.set_option("row_chains", 1)
    eng.set_option("split_route", 1)
    ref = eng.sample_loop(rows, x_cond=x_cond, seed=13, record=(False, True))
    ref = [ref[0].clone(), ref[4].clone()]
    eng.set_option("split_route", 3)
    for chains in (1, 3):
        eng.set_option("row_chains", chains)
        for graph in (False, True):
            got = eng.sample_loop(rows, x_cond=x_cond, seed=13, graph=graph, record=(False, True))
            torch.cuda.synchronize()
            assert eng.get_option("last_chains") == min(chains, (rows + 31) // 32)
            assert torch.equal(got[0], ref[0]) and torch.equal(got[4], ref[1]), (cfg, chains, graph)
    assert eng.status(rows) == 0


def test_split_route_shard_equals_full_batch(cuda):
    """A shard small enough for the split route (400 rows at row0 = 1600, as one rank of an
    8-GPU strong-scaling run of config 2) reproduces those rows of the full 3,200-row batch on
    the one-kernel route bitwise: the route follows the shard size without changing results."""
    from bench import build_config

    d, x_cond, rows = build_config("amass16", cuda, T=10)
    eng = d.engine
    eng.set_option("split_route", 1)
    full = eng.sample_loop(rows, x_cond=x_cond, seed=9)[0].clone()
    eng.set_option("split_route", 0)
    per = rows // x_cond.shape[0]
    s0, n = 1600, 400
    part = eng.sample_loop(n, x_cond=x_cond[s0 // per:(s0 + n) // per], seed=9, row0=s0)[0]
    torch.cuda.synchronize()
    assert torch.equal(part, full[s0:s0 + n])


def test_exact_variant_row_chains_bitwise(cuda):
    """The exact-f32 kernels (v3, LDS-DMA stages) with three concurrent row chains, graph replay,
    equal one chain run eagerly bit for bit (config 2, T = 10)."""
    from bench import build_config

    d, x_cond, rows = build_config("amass16", cuda, T=10)
    eng = d.engine
    eng.set_option("kernel_variant", 3)
    eng.set_option("row_chains", 1)
    ref = eng.sample_loop(rows, x_cond=x_cond, seed=21)[0].clone()
    eng.set_option("row_chains", 3)
    for graph in (False, True, True):
        x = eng.sample_loop(rows, x_cond=x_cond, seed=21, graph=graph)[0]
        torch.cuda.synchronize()
        assert eng.get_option("last_chains") == 3
        assert torch.equal(x, ref), graph


def test_split_route_row_chains_deterministic(cuda):
    """The small-batch split route (k_gl4y + k_gl4 MODE 2 / 3; 200 rows at T = 100) on three row
    chains: repeated runs, eager and graph, are bitwise identical and equal one chain."""
    from bench import build_config

    d, x_cond, rows = build_config("amass16", cuda, T=100, batch=4)
    eng = d.engine
    eng.set_option("row_chains", 1)
    ref = eng.sample_loop(rows, x_cond=x_cond, seed=5)[0].clone()
    eng.set_option("row_chains", 3)
    for graph in (False, False, True, True):
        x = eng.sample_loop(rows, x_cond=x_cond, seed=5, graph=graph)[0]
        torch.cuda.synchronize()
        assert eng.get_option("last_chains") == 3
        assert torch.equal(x, ref), graph


@pytest.mark.parametrize("name", ["release_h36m16_T10", "release_amass21_T10"])
def test_denoiser_per_layer_activations(name, cuda):
    """Every block output of one Denoiser forward (init_lin, 8 ResnetBlocks, 7 attention blocks +
    the final Identity, final_res_block) against the reference's forward hooks."""
    z = golden(name)
    d = build_release_diffusion(z, cuda)
    xcs, fu, start, _ = release_inputs(z)
    x0, acts = d.engine.denoiser_trace(start.to(cuda), int(z["T"]) - 1, xcs.to(cuda))
    names = ["init_lin"] + [f"layer{i}_{k}" for i in range(8) for k in ("res", "attn")] + ["final_res"]
    assert len(acts) == len(names)
    for n, a in zip(names, acts):
        assert _max_err(a, z["act_" + n]) < 1e-5, n
    assert _max_err(x0, z["fwd_x0"]) < 1e-5


@pytest.mark.parametrize("case", ["noattn", "tanh", "timages", "interp"])
def test_sample_surface_variants(case, cuda):
    z = golden("variants_h36m16_T10")
    kw = {}
    if case == "noattn":
        kw = dict(use_attention=False)
    elif case == "tanh":
        kw = dict(final_scale=8.0, diffusion_activation="tanh")
    d = build_release_diffusion(z, cuda, **kw)
    xc, start, samp, noise2 = (t.to(cuda) for t in variant_inputs(z))
    B = start.shape[0]
    if case == "timages":
        img, (_, timgs) = d.sample(batch_size=B, x_cond=xc, start_noise=start, sampling_noise=samp,
                                   return_timages=True)
        assert _max_err(img, z["timages_img"]) < TOL and _max_err(timgs, z["timages"]) < TOL
        img2, (_, nt, timgs2) = d.sample(batch_size=B, x_cond=xc, start_noise=start, sampling_noise=samp,
                                         return_sampling_noise=True, return_timages=True)
        assert torch.equal(img, img2) and torch.equal(timgs, timgs2) and torch.equal(nt, samp)
        return
    if case == "interp":
        img, _ = d.sample(batch_size=B, x_cond=xc, start_noise=start, sampling_noise=samp, if_interpolate=True,
                          noise2interpolate=noise2, interpolation_kwargs={"interpolate_funct": interpolate_funct})
        assert _max_err(img, z["interp_img"]) < TOL
        return
    img, (_, _, mean_t) = d.sample(batch_size=B, x_cond=xc, start_noise=start, sampling_noise=samp,
                                   return_sampling_noise=True)
    assert _max_err(img, z[f"{case}_img"]) < TOL and _max_err(mean_t, z[f"{case}_mean_t"]) < TOL
    if case == "noattn":
        assert sorted(d.state_dict().keys()) == sorted(z["noattn_keys"].tolist())


def test_two_plans_with_different_options_concurrently(cuda):
    """Kernel options are plan state (sd_plan_set_option), not process globals: plan A (auto
    kernels, 3 row chains -- checked by SD_OPT_LAST_CHAINS) and plan B (exact-f32 v3, 1 chain,
    register staging) sample at the same time on two streams from two threads; each equals its
    own solo result bitwise, and the two agree within the split-f16 vs exact-f32 difference."""
    z = golden("release_h36m16_T100")
    da = build_release_diffusion(z, cuda)
    db = build_release_diffusion(z, cuda)
    db.engine.set_option("kernel_variant", 3)
    db.engine.set_option("gl4_staging", 1)
    db.engine.set_option("row_chains", 1)
    da.engine.set_option("row_chains", 3)
    xcs = torch.from_numpy(np.repeat(release_inputs(z)[0].numpy(), 64, 0)).to(cuda)[:64]  # 64 sequences
    rows = 64 * 4
    # no synchronisation: the threads' streams start while these solo runs may still be running
    # on the default stream -- each (plan, stream) pair has its own workspace
    solo_a = da.sample(batch_size=rows, x_cond=xcs, seed=8)[0].clone()
    solo_b = db.sample(batch_size=rows, x_cond=xcs, seed=8)[0].clone()
    res = {}

    def run(name, d):
        s = torch.cuda.Stream(cuda)
        with torch.cuda.stream(s):
            for _ in range(3):
                res[name] = d.sample(batch_size=rows, x_cond=xcs, seed=8)[0]
        s.synchronize()

    th = [threading.Thread(target=run, args=("a", da)), threading.Thread(target=run, args=("b", db))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    assert torch.equal(res["a"], solo_a), _max_err(res["a"], solo_a)
    assert torch.equal(res["b"], solo_b), _max_err(res["b"], solo_b)
    assert _max_err(solo_a, solo_b) < TOL
    assert da.engine.get_option("kernel_variant") == 0 and db.engine.get_option("kernel_variant") == 3
    assert da.engine.get_option("last_chains") == 3 and db.engine.get_option("last_chains") == 1


@pytest.mark.parametrize("cfg,batch", [("freeman17", 64), ("amass16", 8)])
def test_two_default_plans_concurrently(cfg, batch, cuda):
    """Two plans with DEFAULT options sampling at the same time from two threads on two streams
    (ADVICE r02): at J = 17 full batch (tiled split route, 3 chains each) and at 400 rows (k_gl4y
    split route): every kernel of one call may share CUs with the other call's; each result equals
    its solo run bitwise."""
    from bench import build_config

    da, xa, rows = build_config(cfg, cuda, T=10, batch=batch)
    db, xb, _ = build_config(cfg, cuda, T=10, batch=batch, seq0=batch)
    solo = {"a": da.engine.sample_loop(rows, x_cond=xa, seed=1)[0].clone(),
            "b": db.engine.sample_loop(rows, x_cond=xb, seed=2)[0].clone()}
    torch.cuda.synchronize()
    res = {}

    def run(name, d, x, seed):
        s = torch.cuda.Stream(cuda)
        with torch.cuda.stream(s):
            for _ in range(4):
                res[name] = d.engine.sample_loop(rows, x_cond=x, seed=seed)[0]
        s.synchronize()

    th = [threading.Thread(target=run, args=("a", da, xa, 1)), threading.Thread(target=run, args=("b", db, xb, 2))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    for k in ("a", "b"):
        assert torch.equal(res[k], solo[k]), (k, _max_err(res[k], solo[k]))
    assert da.engine.get_option("last_chains") == (3 if rows > 1200 else 2)  # auto row chains


def test_graph_linear_rejects_aliased_output(cuda):
    """A graph-linear launch whose input is its output would race between column tiles (ADVICE
    r01): the library refuses it instead of computing garbage."""
    L = _lib.lib()
    J, K, N, B = 16, 192, 192, 64
    x = torch.randn((B, J, K), device=cuda)
    W = torch.randn((1, N, K), device=cuda) * 0.05
    gh = torch.eye(J, device=cuda)
    types = (torch.zeros(J, dtype=torch.int64)).numpy()
    import ctypes

    tarr = (ctypes.c_int64 * J)(*types.tolist())
    rc = L.sd_test_graph_linear(x.data_ptr(), K, 1, None, 0, W.data_ptr(), None, tarr, gh.data_ptr(), None, 0, None,
                                x.data_ptr(), B, J, N, 0, torch.cuda.current_stream().cuda_stream)
    assert rc != 0 and b"invalid" in L.sd_last_error().lower()


F16_RANGE_CASES = {  # name -> (plan options, Denoiser attention heads / dim per head, precision)
    "auto": ({}, (8, 32), "f32"), "split1_one_kernel": ({"split_route": 1}, (8, 32), "f32"),
    "split2": ({"split_route": 2}, (8, 32), "f32"), "split3": ({"split_route": 3}, (8, 32), "f32"),
    "tile813_one_kernel": ({"gl4_tile": 813}, (8, 32), "f32"),
    # attn_dim_head = 64: no fused to_qkv + attention tile, row-major activations, separate k_attention
    "dh64": ({}, (4, 64), "f32"), "dh64_split1": ({"split_route": 1}, (4, 64), "f32"),
    # half precision's J = 16 full-batch route is the one-kernel tile; here the auto route at 8 rows
    "half_split1": ({"split_route": 1}, (8, 32), "half"),
}


@pytest.mark.parametrize("case", list(F16_RANGE_CASES))
def test_f16_range_exact_in_kernel(case, cuda):
    """Activations the split-f16 products cannot represent (|x| >= 65504; conditioning latents
    scaled by 1e5 and 3e9) on every split-f16 route -- auto, the one-kernel tiles (split_route 1,
    a gl4_tile option), k_gl4y + MODE 2 / 3, tiled k_gl4t + MODE 2 / 3, a Denoiser with
    attn_dim_head = 64 (no fused attention tile) -- with no warning and no host re-run: the waves
    that leave the range recompute their tiles on exact-f32 MFMA in the kernel (exact_tile_f32, in
    the one-kernel tiles too since round 6); the status word records that the fallback ran (in
    range it stays clear).
    Accuracy: at these magnitudes any f32 evaluation order moves the latents by ~1e-3 (an f32 ulp
    of a 1e5 activation is 8e-3, and x0 = clamp(out) passes the rows near +-1 through), so the
    bar is the float64 oracle: sample()'s deviation from it must stay within that of an exact-f32
    plan (kernel variant 3), i.e. f32-accurate.  In range the 1e-4 latent bar holds (goldens).
    Half precision: its in-range tiles are one f16 product (not f32-accurate by definition); the
    out-of-range tiles are recomputed exactly, so the latents stay finite."""
    import dataclasses
    import warnings

    opts, (heads, dh), prec = F16_RANGE_CASES[case]
    z = golden("release_h36m16_T10")
    d = build_release_diffusion(z, cuda, attn_heads=heads, attn_dim_head=dh)
    if prec != "f32":
        d.engine.set_precision(prec)
    for k, v in opts.items():
        d.engine.set_option(k, v)
    xcs, fu, start, samp = release_inputs(z)
    kw = dict(batch_size=start.shape[0], start_noise=start.to(cuda), sampling_noise=samp.to(cuda))
    d.sample(x_cond=xcs.to(cuda), **kw)
    assert d.engine.status(start.shape[0]) == 0
    route = d.engine.get_option("last_route")
    if "one_kernel" in case:
        assert route & 3, route  # k_gl4 MODE 0 / 1 ran
    ref = build_release_diffusion(z, cuda, attn_heads=heads, attn_dim_head=dh)
    ref.engine.set_option("kernel_variant", 3)
    sd, cfg, bufs = _oracle_setup(d)
    cfg = dataclasses.replace(cfg, heads=heads, dim_head=dh)
    sd64 = {k: v.double() if v.is_floating_point() else v for k, v in sd.items()}
    bufs64 = {k: v.double() if v.is_floating_point() else v for k, v in bufs.items()}
    for scale in (1e5, 3e9):
        big = xcs * scale
        with warnings.catch_warnings():
            warnings.simplefilter("error")
            img = d.sample(x_cond=big.to(cuda), **kw)[0]
            torch.cuda.synchronize()
        assert d.engine.status(start.shape[0]) & _lib.SD_STATUS_F16_RANGE
        assert torch.isfinite(img).all()
        if prec != "f32":
            continue
        img_exact = ref.sample(x_cond=big.to(cuda), **kw)[0]
        img64, _ = O.p_sample_loop(sd64, cfg, bufs64, start.double(), samp.double(), x_cond=big.double())
        err, err_exact = _max_err(img, img64), _max_err(img_exact, img64)
        assert err <= max(1.5 * err_exact, TOL), (case, scale, err, err_exact)
