#!/usr/bin/env python3
"""Headline benchmark: generated futures/sec of NonisotropicGaussianDiffusion.sample() on the
MI355X HIP engine (BASELINE.json metric), one process per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config amass16] [--scaling weak|strong]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

A "step" is one full sample() call: the T-step reverse chain over one batch of
`batch` sequences x `futures` futures (B rows), with the release Denoiser and device Philox
noise, inputs resident in HBM.  Ranks shard whole sequences (row0 = the rank's first global row,
so the device noise and the outputs do not depend on the GPU count); there is no collective in
the data path.  --scaling weak (default): every rank samples `batch` sequences (per-GPU work
fixed as N grows); --scaling strong: the `batch` sequences are split over the N ranks
(sharded.shard_range), total work fixed.  Weights are the repo's deterministic synthetic filler
(no checkpoint can be fetched); conditioning latents are synthetic U(-1, 1).

Rank 0 prints one JSON line.  It also carries:
  roofline      the dominant kernel class: one graph-linear layer (on the split routes its GEMM
                phase + mixing / attention phase; fused to_qkv + attention launches included),
                >= 97 % of a denoise step's kernel time.  Bound "hbm": achieved = the layer's
                algorithmic HBM bytes (activations in and out once, residual in, weights once)
                per launch / its average duration, timed with HIP events on the launch stream
                (sd_profile_step, one denoise step at the full batch; rocprofv3 --kernel-trace of
                the same command under profiles/ gives the per-kernel durations) vs 8 TB/s;
                traffic = PMC HBM bytes per layer launch (FETCH_SIZE x 2 + WRITE_SIZE, separate
                passes, profiles/pmc_traffic.json keyed by config and the kernels the call
                launched).  "mfma_view" prices the same launches by their f32 FLOPs against the
                f16 MFMA peak / 3 (2500 / 3 TFLOP/s: every f32 product is three f16 products);
                "timed_region" by the FLOPs of the whole timed step (row chains, hipGraphs, the
                update kernels and launch gaps inside) / ms_per_step;
  exact_f32     (N = 1) the same workload on the exact-f32 kernels (kernel_variant 3);
  cpu_baseline  the oracle (torch-CPU restatement of the reference path) on this host's physical
                cores (those this process may use: affinity and cgroup quota), median of 3 runs
                of a few of the T steps on the same B rows, per-step time x T.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from skeletondiffusion_amd import _lib, synthetic  # noqa: E402
from skeletondiffusion_amd.core.diffusion import NonisotropicGaussianDiffusion, get_cov_from_corr  # noqa: E402
from skeletondiffusion_amd.core.network import Denoiser  # noqa: E402
from skeletondiffusion_amd.skeletons import skeleton  # noqa: E402

METRIC = "generated futures/sec (AMASS 16-joint, 50 futures, T=100) at 1/2/4/8 GPUs"
FP32_PEAK_TFLOPS = 157.3   # MI355X fp32 dense (vector = matrix), MI355X_MICROARCH.md
F16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X f16/bf16 dense MFMA (no sparsity), MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec

# BASELINE.json configs -> (skeleton, T, batch sequences, futures)
CONFIGS = {
    "amass16": dict(skel="h36m16", T=100, batch=64, futures=50,
                    workload="AMASS 16-joint nonisotropic sampling, T=100, 50 futures, batch=64 (config 2)"),
    "amass21": dict(skel="amass21", T=100, batch=64, futures=50,
                    workload="AMASS real node count J=21, T=100, 50 futures, batch=64 (config 2, secondary)"),
    "mano51": dict(skel="mano51", T=100, batch=64, futures=50,
                   workload="AMASS-MANO J=51, T=100, 50 futures, 64 sequences per GPU (config 3 per-rank shard)"),
    "mano52": dict(skel="mano52", T=100, batch=64, futures=50,
                   workload="AMASS-MANO hip-included J=52, T=100, 50 futures, 64 sequences per GPU (config 3 label)"),
    "h36m_t1000": dict(skel="h36m16", T=1000, batch=1, futures=50,
                       workload="Human3.6M J=16, T=1000, 50 futures, 1 sequence, hipGraph (config 4)"),
    "freeman17": dict(skel="freeman17", T=100, batch=64, futures=50,
                      workload="FreeMan J=17, T=100, 50 futures, batch=64, fp32 (config 5 shape)"),
    # config 5 as BASELINE.json states it: 11,015 test sequences x 50 futures over 8 GPUs (1,377 per
    # GPU), T=10 (release), reduced precision (here: the half mode, one f16 product per MAC)
    "freeman17_half": dict(skel="freeman17", T=10, batch=1377, futures=50, precision="half",
                           workload="FreeMan J=17, T=10, 50 futures, 1,377 sequences per GPU, half precision "
                                    "(f16 products, f32 activations)"),
    # config 5 as stated: bf16 latents + fp32 Sigma_N projection
    "freeman17_bf16": dict(skel="freeman17", T=10, batch=1377, futures=50, precision="bf16",
                           workload="FreeMan J=17, T=10, 50 futures, 1,377 sequences per GPU (11,015 over 8 GPUs), "
                                    "bf16 latents + fp32 Sigma_N projection (config 5)"),
}

RELEASE_ARCH = dict(use_attention=True, self_condition=False, norm_type="none", depth=4, attn_dim_head=32,
                    attn_heads=8, learn_influence=True)


def skeleton_covariance(skel, adj):
    """(Sigma_N, Lambda_N, U) for a skeleton.  In deployment these are checkpoint buffers; here the
    values the reference computed in the build container (tests/golden/cov_<skel>.npz) are used,
    because eigh on another LAPACK build may pick other eigenvector signs / degenerate-eigenspace
    bases (and for MANO the reference's own PD assert fails on the GPU box's LAPACK)."""
    path = os.path.join(HERE, "tests", "golden", f"cov_{skel}.npz")
    if os.path.exists(path):
        z = np.load(path)
        return tuple(torch.from_numpy(z[k]) for k in ("Sigma_N", "Lambda_N", "U"))
    return get_cov_from_corr(torch.from_numpy(adj), if_sigma_n_scale=True, sigma_n_scale="spectral")


def build_config(name, device, T=None, batch=None, futures=None, seed=1234, seq0=0):
    """Release-architecture diffusion with synthetic weights + per-sequence conditioning latents.
    Returns (diffusion on `device`, x_cond (batch, J, 96) on `device`, rows = batch * futures)."""
    c = CONFIGS[name]
    T = T or c["T"]
    batch = batch or c["batch"]
    futures = futures or c["futures"]
    _, _, adj, types = skeleton(c["skel"])
    J = adj.shape[0]
    m = Denoiser(dim=96, cond_dim=96, out_dim=96, channels=J, num_nodes=J, node_types=torch.from_numpy(types),
                 **RELEASE_ARCH)
    synthetic.fill_module_(m, seed)
    S, L, U = skeleton_covariance(c["skel"], adj)
    d = NonisotropicGaussianDiffusion(Sigma_N=S, Lambda_N=L, U=U, model=m, latent_size=96, diffusion_timesteps=T,
                                      diffusion_objective="pred_x0", diffusion_conditioning=True,
                                      beta_schedule="cosine").to(device).eval()
    # sequence s gets its own conditioning latent (seeded by its global index)
    xc = np.stack([synthetic.uniform((J, 96), 10_000 + seq0 + s) for s in range(batch)])
    return d, torch.from_numpy(xc).to(device), batch * futures


def shard(rank: int, batch: int, futures: int, world: int = 1, scaling: str = "weak"):
    """Shard of rank `rank`, all futures of a sequence on one rank (eval_prepare_model.py:96
    repeat_interleave order).  weak: sequences [rank*batch, (rank+1)*batch); strong: rank's
    balanced part of the `batch` sequences (sharded.shard_range).
    Returns (seq0, row0, rows); row0 keys the device noise so outputs are GPU-count invariant."""
    if scaling == "strong":
        from skeletondiffusion_amd.sharded import shard_range

        s0, s1 = shard_range(batch, rank, world)
        return s0, s0 * futures, (s1 - s0) * futures
    return rank * batch, rank * batch * futures, batch * futures


def graph_linear_bytes(d, rows, fused_attn):
    """Algorithmic HBM bytes of one denoise step's graph-linear launches: every activation read
    once and written once (f32), every weight read once (f32 or split f16 pair: 4 B either way)."""
    m = d.model
    J, H = d.channels, m.dim + m.cond_dim
    hid = m.attn_heads * m.attn_dim_head if hasattr(m, "attn_heads") else 256
    total = 0.0
    for mod in m.modules():
        if type(mod).__name__ != "StaticGraphLinear":
            continue
        N, K = mod.weight.shape[-2], mod.weight.shape[-1]
        fused_qkv = fused_attn and N == 3 * hid
        out_n = hid if fused_qkv else N
        total += 4.0 * rows * J * (K + out_n) + 4.0 * mod.weight.numel()
    # residual reads: every ResnetBlock's block2 and every attention's to_out add a (B, J, H) residual
    n_res = sum(type(mod).__name__ in ("ResnetBlock", "Attention") for mod in m.modules())
    total += 4.0 * rows * J * H * n_res
    return total


def profile_kernels(d, x_cond, rows, reps=5):
    eng = d.engine
    plan = eng.plan()
    L = _lib.lib()
    J, D, T = d.channels, d.seq_length, d.num_timesteps
    x = torch.randn((rows, J, D), device=x_cond.device, generator=torch.Generator(x_cond.device).manual_seed(3))
    ws, nb = eng.workspace(rows)
    ms = (ctypes.c_float * 4)()
    cnt = (ctypes.c_int32 * 3)()
    stream = torch.cuda.current_stream(x_cond.device).cuda_stream
    rep = rows // x_cond.shape[0]
    _lib.check(L.sd_profile_step(plan, x.data_ptr(), x_cond.data_ptr(), rep, T // 2, rows, ws.data_ptr(), nb, 1,
                                 ms, cnt, stream))  # warm
    _lib.check(L.sd_profile_step(plan, x.data_ptr(), x_cond.data_ptr(), rep, T // 2, rows, ws.data_ptr(), nb, reps,
                                 ms, cnt, stream))
    fl = (ctypes.c_double * 3)()
    _lib.check(L.sd_plan_step_flops(plan, rows, fl))
    return list(ms), list(cnt), list(fl)


def host_cpu():
    """lscpu-style description of this host's CPU (model, sockets x cores x threads)."""
    info = {}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            info[k.strip()] = v.strip()
    except Exception:
        pass
    return {"model": info.get("Model name", "unknown"), "sockets": info.get("Socket(s)"),
            "cores_per_socket": info.get("Core(s) per socket"), "threads_per_core": info.get("Thread(s) per core"),
            "logical_cpus": os.cpu_count()}


def physical_cores():
    """Physical cores this process may run on: lscpu's sockets x cores per socket, capped by the
    CPU affinity mask (logical CPUs / threads per core) and the cgroup CPU quota (cpu.max)."""
    h = host_cpu()
    try:
        phys = int(h["sockets"]) * int(h["cores_per_socket"])
        tpc = max(1, int(h["threads_per_core"]))
    except (TypeError, ValueError):
        phys, tpc = os.cpu_count() or 1, 1
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(float(q) / float(period)))
    except Exception:
        pass
    n = min(phys, max(1, avail // tpc) if avail < (os.cpu_count() or avail) else phys)
    if quota:
        n = min(n, quota)
    return max(1, n), {"physical_cores": phys, "threads_per_core": tpc, "affinity_cpus": avail, "cgroup_cpu_quota": quota}


def cpu_baseline(d, x_cond, rows, steps, threads, repeats=3):
    """The oracle (torch-CPU restatement of the reference path) on a bounded sample: one warm-up
    step, then the median of `repeats` timed runs of `steps` reverse steps."""
    import oracle as O

    torch.set_num_threads(threads)
    J, D, T = d.channels, d.seq_length, d.num_timesteps
    sd = {k: v.detach().cpu() for k, v in d.state_dict().items()}
    cfg = O.release_config(J, d.model.node_types)
    bufs = {k: v for k, v in sd.items() if not k.startswith("model.")}
    xc = x_cond.cpu()
    g = torch.Generator().manual_seed(0)
    start = torch.randn((rows, J, D), generator=g)
    O.p_sample_loop(sd, cfg, bufs, start, None, x_cond=xc, steps=1)   # warm-up step
    runs = []
    for _ in range(repeats):
        t0 = time.perf_counter()
        O.p_sample_loop(sd, cfg, bufs, start, None, x_cond=xc, steps=steps)
        runs.append((time.perf_counter() - t0) / steps)
    per_step = float(np.median(runs))
    return {"value": rows / (per_step * T), "unit": "futures/s", "cores": threads, "kind": "port",
            "host_cpu": host_cpu(), "runs_futures_per_s": [rows / (r * T) for r in runs],
            "sample": f"oracle/skeldiff_oracle.py p_sample_loop, median of {repeats} runs of {steps} of the T={T} "
                      f"reverse steps on the same {rows} rows (J={J}), per-step time x T; torch-CPU fp32, "
                      f"{threads} threads (torch.set_num_threads)"}


def world_rows(world: int, rows: int, scaling: str, batch: int, futures: int) -> int:
    """Rows all ranks process per step: weak = world x this rank's rows; strong = the batch."""
    return batch * futures if scaling == "strong" else world * rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="amass16", choices=sorted(CONFIGS))
    ap.add_argument("--T", type=int, default=None)
    ap.add_argument("--batch", type=int, default=None, help="sequences per GPU")
    ap.add_argument("--futures", type=int, default=None)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--precision", choices=["f32", "half", "bf16"], default=None,
                    help="graph-linear arithmetic (default: the config's; f32 for the BASELINE metric)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=4)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: every physical core this process may use")
    ap.add_argument("--profile-reps", type=int, default=5)
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak",
                    help="weak: `batch` sequences per GPU; strong: `batch` sequences split over the GPUs")
    ap.add_argument("--kernel-variant", type=int, default=0, help="0 auto (split-f16 v4), 3 exact f32, ...")
    ap.add_argument("--no-exact-line", action="store_true", help="skip the exact-f32 comparison (N=1)")
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                    help="per-plan kernel option (engine.set_option), e.g. split_route=3, row_chains=1")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # one rank per GPU; the modulo only matters for a rehearsal with more ranks than GPUs
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        # "nccl" = RCCL over xGMI; SKELDIFF_DIST_BACKEND=gloo rehearses the multi-rank path on one GPU
        backend = os.environ.get("SKELDIFF_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    c = CONFIGS[args.config]
    batch = args.batch or c["batch"]
    futures = args.futures or c["futures"]
    seq0, row0, rows = shard(rank, batch, futures, world, args.scaling)
    nseq_local = rows // futures
    d, x_cond, rows = build_config(args.config, dev, T=args.T, batch=nseq_local, futures=futures, seq0=seq0)
    J, D, T = d.channels, d.seq_length, d.num_timesteps
    if dist:  # every rank samples with rank 0's parameters (RCCL broadcast over xGMI, untimed setup)
        from skeletondiffusion_amd.sharded import broadcast_state
        broadcast_state(d)
    eng = d.engine
    eng.set_precision(args.precision or c.get("precision", "f32"))
    eng.set_option("kernel_variant", args.kernel_variant)
    for o in args.option:
        name, value = o.split("=", 1)
        eng.set_option(name, int(value))
    eng.plan()
    graph = not args.no_graph
    stream = torch.cuda.Stream(dev)
    out = torch.empty((rows, J, D), device=dev)
    base_seed = 20251015

    eng.enable_graph(graph)

    def step(i):
        # the metric's definition: wall time of the public NonisotropicGaussianDiffusion.sample()
        # (base.py:439-443 -> p_sample_loop -> torch.ops.skeldiff.sample_loop), output buffer reused
        d.sample(batch_size=rows, x_cond=x_cond, seed=base_seed + i, row0=row0, out=out)

    with torch.cuda.stream(stream):
        for i in range(args.warmup):
            step(10_000 + i)
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(args.steps):
            step(i)
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
        torch.cuda.synchronize(dev)
        elapsed = time.perf_counter() - t0
        # what the timed calls ran (read before the profiling / exact-f32 calls below)
        row_chains = eng.get_option("last_chains")
        route_bits = eng.get_option("last_route")
        assert torch.isfinite(out).all(), "non-finite latents"
        if dist:
            tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            elapsed = float(tt.item())
        ms, cnt, fl = profile_kernels(d, x_cond, rows, args.profile_reps)
        exact = None
        if (world == 1 and not args.no_exact_line and args.kernel_variant == 0 and J in (16, 17, 21)
                and eng.precision == "f32"):
            # the same workload on the exact-f32 kernels: a second plan, same inputs
            eng.set_option("kernel_variant", 3)
            for i in range(args.warmup):
                step(20_000 + i)
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            for i in range(args.steps):
                step(i)
            torch.cuda.synchronize(dev)
            el3 = time.perf_counter() - t1
            eng.set_option("kernel_variant", args.kernel_variant)
            exact = {"value": rows * args.steps / el3, "unit": "futures/s", "ms_per_step": el3 / args.steps * 1e3,
                     "kernels": "exact f32 (kernel_variant 3: k_gl3 / k_gl2 on v_mfma_f32_32x32x2_f32, "
                                "separate k_attention)",
                     "graph_linear_tflops_timed": None}

    value = world_rows(world, rows, args.scaling, batch, futures) * args.steps / elapsed
    variant = eng.get_option("kernel_variant")
    kernels = [name for bit, name in sorted(_lib.ROUTE_BITS.items()) if route_bits & bit]
    split = bool(route_bits & (1 | 2 | 4 | 8)) and not (route_bits & 64)  # split-f16 products (v4 / v5 GEMM phase)
    tiled = bool(route_bits & 8) and J <= 21
    small = bool(route_bits & 4)
    route = ("tiled split (k_gl4t + k_gl4 MODE 2/3)" if tiled and not route_bits & (1 | 2) else
             "tiled split + one-kernel fused attention" if tiled else
             "small-batch split (k_gl4y + k_gl4 MODE 2/3)" if small else
             "v5 (k_gl4t + k_gl5_mixd + k_attention_mix)" if route_bits & 32 and route_bits & 1024 and split else
             "v5 (k_gl4t + k_gl5_mixd + k_attention)" if route_bits & 32 and split else
             "one-kernel (k_gl4)" if split else "exact f32")
    half = split and eng.precision in ("half", "bf16")
    # the to_qkv layer's mixing inside the attention launch (k_attention_mix): to_qkv + attention
    # count as one fused layer (its bytes, FLOPs and both launches' time), as on the fused routes
    attn_mix = bool(route_bits & 1024)
    fused_attn = (ms[1] == 0.0 and cnt[1] == 0) or attn_mix  # attention inside the layer's launches
    gl_ms = ms[0] + (ms[1] if attn_mix else 0.0)
    gl_flops = fl[0] + (fl[1] if fused_attn else 0.0)
    gl_tflops = gl_flops / (gl_ms * 1e-3) / 1e12
    peak = F16_MFMA_PEAK_TFLOPS if half else F16_MFMA_PEAK_TFLOPS / 3.0 if split else FP32_PEAK_TFLOPS
    gl_bytes = graph_linear_bytes(d, rows, fused_attn)
    gl_gbs = gl_bytes / (gl_ms * 1e-3) / 1e9
    launches = max(cnt[0], 1)
    upd_bytes = 3.0 * rows * J * D * 4        # x0, x_t in, x_{t-1} out (device Philox noise)
    upd_gbs = upd_bytes / (ms[2] * 1e-3) / 1e9
    step_flops = sum(fl)
    ms_step = elapsed / args.steps * 1e3
    # graph-linear work of the timed region: T denoise steps per bench step, on this rank's rows
    timed_tflops = (fl[0] + fl[1]) * T / (ms_step * 1e-3) / 1e12
    if exact is not None:
        exact["graph_linear_tflops_timed"] = (fl[0] + fl[1]) * T / (exact["ms_per_step"] * 1e-3) / 1e12
        exact["frac_of_f32_peak"] = exact["graph_linear_tflops_timed"] / FP32_PEAK_TFLOPS
    traffic, traffic_note = None, "no PMC pass on record for this config and kernel set"
    traffic_file = os.path.join(HERE, "profiles", "pmc_traffic.json")
    traffic_key = f"{args.config}|{route_bits}"
    if os.path.exists(traffic_file):
        try:
            tr = json.load(open(traffic_file)).get(traffic_key)
            if tr and tr.get("rows") == rows:
                traffic = tr.get("hbm_bytes_per_layer_launch")
                traffic_note = tr.get("source")
        except Exception:
            pass
    rec = {
        "metric": METRIC,
        "value": value,
        "unit": "futures/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": ("bf16" if eng.precision == "bf16" else "f16") if half else
                 "f32 (emulated: 3 x f16 split products)" if split else "f32",
        "arithmetic": ("bf16: one bf16 product per multiply-add on v_mfma_f32_32x32x16_bf16, f32 accumulate; "
                       "bf16 latents and residual-stream activations in HBM; f32 posterior update (Sigma_N / U "
                       "projections); latent ADE/APD within 1 % of the oracle (tests/test_precision.py)")
        if half and eng.precision == "bf16" else
        ("half: one f16 product per multiply-add on v_mfma_f32_32x32x16_f16, f32 accumulate, f32 "
         "activations in HBM (latent ADE/APD within 1 % of the f32 mode, tests/test_precision.py)")
        if half else ("f32-accurate: 3 x f16 split products on v_mfma_f32_32x32x16_f16, f32 accumulate "
                       "(end-to-end error within the f32-vs-f64 drift, tools/sim_split_f16.py); "
                       "exact-f32 kernels via SKELDIFF_GL_VARIANT=3") if split else "exact f32 (f32 MFMA)",
        "data": "synthetic (deterministic synthetic weights of the release Denoiser; U(-1,1) conditioning "
                "latents; device Philox noise)",
        "config": {"workload": c["workload"], "J": J, "T": T, "sequences_per_gpu": rows // futures,
                   "sequences_total": world_rows(world, rows, args.scaling, batch, futures) // futures,
                   "futures": futures, "rows_per_gpu": rows, "latent_dim": D, "hipgraph": graph,
                   "parallelism": f"dp{world} (sequence-sharded, no data-path collective)",
                   "row_chains": row_chains, "route": route, "kernels": kernels, "route_bits": route_bits,
                   "kernel_variant": variant},
        "roofline": {
            "bound": "hbm",
            "kernel": "one graph-linear layer: " + route + " (the launches of one StaticGraphLinear, to_qkv + "
                      "attention fused); per-launch average over the layers of one denoise step",
            "achieved": gl_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gl_gbs / HBM_PEAK_GBS,
            "traffic": traffic, "traffic_source": traffic_note,
            "algorithmic_bytes_per_launch": gl_bytes / launches, "avg_launch_ms": gl_ms / launches,
            "launches_per_denoise_step": cnt[0],
            "measured_on": ("HIP events on the launch stream around each layer, one denoise step at the full "
                            "batch on one stream (sd_profile_step, kernels alone on the GPU), "
                            f"{args.profile_reps} repetitions"),
            "mfma_view": {"achieved": gl_tflops, "peak": peak, "unit": "TFLOP/s", "frac": gl_tflops / peak,
                          "flops_per_launch": gl_flops / launches,
                          "peak_basis": "f16 / bf16 dense MFMA 2500 TFLOP/s (one product per multiply-add)" if half
                          else "f16 dense MFMA 2500 TFLOP/s / 3 products per f32 product" if split
                          else "f32 dense 157.3 TFLOP/s"},
            "timed_region": {"achieved": timed_tflops, "peak": peak, "unit": "TFLOP/s", "frac": timed_tflops / peak,
                             "flops_per_denoise_step": fl[0] + fl[1],
                             "measured_on": "graph-linear + attention FLOPs of T denoise steps over this rank's rows "
                                            "/ ms_per_step (row chains, hipGraphs, update kernels, gaps inside)"},
        },
        "kernels_per_denoise_step_ms": {"graph_linear": ms[0], "attention": ms[1], "update": ms[2],
                                        "step_first_to_last_event": ms[3]},
        "update_kernel": {"bound": "hbm", "achieved": upd_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": upd_gbs / HBM_PEAK_GBS, "bytes_per_launch": upd_bytes,
                          "avg_launch_ms": ms[2] / max(cnt[2], 1)},
        "step_algorithmic_tflops_per_gpu": step_flops * T * args.steps / elapsed / 1e12,
    }
    if exact is not None:
        rec["exact_f32"] = exact
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads, cores = physical_cores()
        rec["cpu_baseline"] = cpu_baseline(d, x_cond, rows, args.cpu_steps, args.cpu_threads or threads)
        rec["cpu_baseline"]["host_cores"] = cores
        rec["speedup_vs_cpu_baseline"] = value / rec["cpu_baseline"]["value"]
    if dist:
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
