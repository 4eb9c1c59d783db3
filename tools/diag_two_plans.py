"""Diagnostic: plan B (exact-f32 v3, 1 chain, register staging) sampled right after plan A."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from conftest import build_release_diffusion, golden, release_inputs  # noqa: E402

cuda = torch.device("cuda:0")
z = golden("release_h36m16_T100")
xcs = torch.from_numpy(np.repeat(release_inputs(z)[0].numpy(), 64, 0)).to(cuda)[:64]
rows = 256


def mk(variant=0, staging=0, chains=3):
    d = build_release_diffusion(z, cuda)
    d.engine.set_option("kernel_variant", variant)
    d.engine.set_option("gl4_staging", staging)
    d.engine.set_option("row_chains", chains)
    return d


def case(mode):
    da = mk()
    db = mk(3, 1, 1)
    a = da.sample(batch_size=rows, x_cond=xcs, seed=8)[0].clone()
    if mode == 1:
        torch.cuda.synchronize()
    if mode == 2:
        db.engine.plan()
        torch.cuda.synchronize()
    b = db.sample(batch_size=rows, x_cond=xcs, seed=8)[0].clone()
    torch.cuda.synchronize()
    b2 = db.sample(batch_size=rows, x_cond=xcs, seed=8)[0].clone()
    torch.cuda.synchronize()
    print(f"mode {mode}: |b - a| {(b - a).abs().max().item():.3g}  |b2 - a| {(b2 - a).abs().max().item():.3g}", flush=True)


for m in (0, 1, 2, 0):
    case(m)
