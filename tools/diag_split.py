"""Split route vs one-kernel route, per Denoiser block output (sd_denoiser_trace): max |diff|."""
import sys

import torch

sys.path.insert(0, ".")
from bench import build_config  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "h36m_t1000"
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 1
dev = torch.device("cuda:0")
d, x_cond, rows = build_config(cfg, dev, T=10, batch=batch)
eng = d.engine
eng.set_option("row_chains", 1)
g = torch.Generator(device="cpu").manual_seed(0)
x = torch.randn((rows, d.channels, d.seq_length), generator=g).to(dev)
res = {}
for sp in (1, 2):
    eng.set_option("split_route", sp)
    x0, acts = eng.denoiser_trace(x, 5, x_cond=x_cond)
    torch.cuda.synchronize()
    res[sp] = [x0.clone()] + [a.clone() for a in acts]
for i, (a, b) in enumerate(zip(res[1], res[2])):
    diff = (a - b).abs()
    print(i, "max", float(diff.max()), "nbad", int((diff > 0).sum()), "of", a.numel(), flush=True)
