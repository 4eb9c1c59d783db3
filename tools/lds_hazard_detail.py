"""where the co-residency differences land.  Config 2 (J=16, B=3200) at T=1
(one denoiser pass + clamp: no chaotic amplification), 1 chain vs 3 chains, many repeats;
prints per run the differing elements, rows, 32-row tiles, magnitude histogram and, for the
first differing row, which nodes / feature ranges differ."""

import sys

import torch

sys.path.insert(0, ".")
from bench import build_config  # noqa: E402
from skeletondiffusion_amd import _lib  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 1
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
staging = int(sys.argv[3]) if len(sys.argv) > 3 else 2  # 2: the diagnostic shared-CU LDS-DMA mode
cuda = torch.device("cuda:0")
d, x_cond, rows = build_config("amass16", cuda, T=T)
d.engine.set_option("gl4_staging", staging)
L = _lib.lib()
g = torch.Generator().manual_seed(5)
start = torch.randn((rows, 16, 96), generator=g).to(cuda)
samp = torch.randn((rows, max(T - 1, 0), 16, 96), generator=g).to(cuda) if T > 1 else None
d.engine.set_option("row_chains", 1)
ref = d.engine.sample_loop(rows, x_cond=x_cond, start_noise=start, sampling_noise=samp, graph=False)[0].clone()
print(f"staging={staging} T={T}", flush=True)
for r in range(reps):
    d.engine.set_option("row_chains", 3)
    a = d.engine.sample_loop(rows, x_cond=x_cond, start_noise=start, sampling_noise=samp, graph=False)[0].clone()
    torch.cuda.synchronize()
    diff = (a - ref).abs()
    nz = diff > 0
    rows_bad = nz.view(rows, -1).any(1)
    tiles = torch.unique(torch.nonzero(rows_bad).flatten() // 32).tolist()
    h = [int(((diff > lo) & (diff <= hi)).sum()) for lo, hi in ((0, 1e-6), (1e-6, 1e-4), (1e-4, 1e-2), (1e-2, 1e9))]
    print(f"rep {r}: {int(nz.sum())} elements, {int(rows_bad.sum())} rows, {len(tiles)} tiles {tiles[:12]}; "
          f"|d| in (0,1e-6]/(1e-6,1e-4]/(1e-4,1e-2]/>1e-2: {h}; max {diff.max().item():.3g}", flush=True)
    if rows_bad.any():
        r0 = int(torch.nonzero(rows_bad)[0])
        m = nz[r0]  # (16, 96)
        nodes = torch.nonzero(m.any(1)).flatten().tolist()
        feats = torch.nonzero(m.any(0)).flatten().tolist()
        print(f"   first bad row {r0}: nodes {nodes}; features {feats[:8]}..{feats[-4:]} ({len(feats)})", flush=True)
