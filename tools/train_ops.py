"""aten-op census of one training step (tools/bench_train.py's step, HIP mode) with
torch.profiler: which torch ops are still launched around the HIP training kernels, how many per
step and their device time.  Usage: python tools/train_ops.py [--J 16] [--rows 1024]"""
import argparse
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from conftest import build_release_diffusion, golden  # noqa: E402
from bench_train import FIX  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--J", type=int, default=16)
    ap.add_argument("--rows", type=int, default=1024)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    z = golden(FIX[a.J])
    T = int(z["T"])
    gen = torch.Generator().manual_seed(1)
    xs = (torch.rand(a.rows, a.J, 96, generator=gen) * 2 - 1).to(dev)
    xc = (torch.rand(a.rows, a.J, 96, generator=gen) * 2 - 1).to(dev)
    d = build_release_diffusion(z, device=dev).train()
    opt = torch.optim.Adam(d.model.parameters(), lr=1e-4)
    g = torch.Generator(device=dev).manual_seed(0)

    def step():
        t = torch.randint(0, T, (a.rows,), device=dev, generator=g)
        loss, _, _ = d.p_losses(xs, t, x_cond=xc)
        opt.zero_grad(set_to_none=True)
        loss.mean().backward()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        step()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="count", row_limit=45))
    print(prof.key_averages(group_by_input_shape=False).table(sort_by="self_device_time_total", row_limit=30))


if __name__ == "__main__":
    main()
