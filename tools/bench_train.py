"""Training-step throughput of the release Denoiser (SURVEY.md §8f "next" #4): one step =
NonisotropicGaussianDiffusion.p_losses (reference base.py:262-300) + backward + Adam update over a
synthetic batch, with the StaticGraphLinears on the HIP training kernels (sd_train.hip) and, for
comparison, on torch ops on the same GPU (training.set_hip_training(False)).  Prints one JSON line.
Usage: python tools/bench_train.py [--J 16] [--rows 1024] [--steps 10] [--warmup 3]"""
import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from conftest import build_release_diffusion, golden  # noqa: E402
from skeletondiffusion_amd import training  # noqa: E402

FIX = {16: "release_h36m16_T10", 21: "release_amass21_T10", 17: "release_freeman17_T10"}


def run(d, xs, xc, T, steps, warmup):
    opt = torch.optim.Adam(d.model.parameters(), lr=1e-4)
    g = torch.Generator(device=xs.device).manual_seed(0)

    def step():
        t = torch.randint(0, T, (xs.shape[0],), device=xs.device, generator=g)
        loss, _, _ = d.p_losses(xs, t, x_cond=xc)
        opt.zero_grad(set_to_none=True)
        loss.mean().backward()
        opt.step()
        return loss

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps, float(loss.mean())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--J", type=int, default=16)
    ap.add_argument("--rows", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--modes", default="hip,torch", help="hip,torch or one of them (profiling)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    z = golden(FIX[a.J])
    T = int(z["T"])
    gen = torch.Generator().manual_seed(1)
    xs = (torch.rand(a.rows, a.J, 96, generator=gen) * 2 - 1).to(dev)
    xc = (torch.rand(a.rows, a.J, 96, generator=gen) * 2 - 1).to(dev)
    res = {}
    for mode in a.modes.split(","):
        training.set_hip_training(mode == "hip")
        d = build_release_diffusion(z, device=dev).train()
        s, loss = run(d, xs, xc, T, a.steps, a.warmup)
        res[mode] = {"ms_per_step": s * 1e3, "samples_per_s": a.rows / s, "last_loss": loss}
        del d
    training.set_hip_training(True)
    print(json.dumps({"metric": "training samples/s (p_losses + backward + Adam)", "J": a.J, "rows": a.rows,
                      "T": T, "data": "synthetic latents, release Denoiser with synthetic weights",
                      "hip": res.get("hip"), "torch_ops_same_gpu": res.get("torch"),
                      "speedup": res["torch"]["ms_per_step"] / res["hip"]["ms_per_step"] if len(res) == 2 else None}))


if __name__ == "__main__":
    main()
