"""Row-chain determinism probe: the config-2 sampler twice per (chains, graph) setting."""
import os
import sys
import torch
sys.path.insert(0, ".")
from bench import build_config
from skeletondiffusion_amd import _lib

cuda = torch.device("cuda:0")
d, x_cond, rows = build_config("amass16", cuda, T=int(sys.argv[1]) if len(sys.argv) > 1 else 100)
L = _lib.lib()
variant = int(os.environ.get("VARIANT", "0"))
L.sd_set_kernel_variant(variant, -1)
L.sd_set_row_chains(1)
ref = d.engine.sample_loop(rows, x_cond=x_cond, seed=11, graph=False)[0].clone()
for graph in [g == "1" for g in os.environ.get("GRAPHS", "0").split()]:
    for n in [int(c) for c in os.environ.get("NCH", "4").split()]:
        L.sd_set_row_chains(n)
        a = d.engine.sample_loop(rows, x_cond=x_cond, seed=11, graph=graph)[0].clone()
        b = d.engine.sample_loop(rows, x_cond=x_cond, seed=11, graph=graph)[0].clone()
        torch.cuda.synchronize()
        da = (a - ref).abs().view(rows, -1).amax(1)
        db = (b - ref).abs().view(rows, -1).amax(1)
        bad_a = torch.nonzero(da).flatten().tolist()
        bad_b = torch.nonzero(db).flatten().tolist()
        print(f"variant={variant} serial={os.environ.get('SKELDIFF_CHAIN_SERIAL')} graph={graph} chains={n}: "
              f"a max {da.max().item():.3g} rows {bad_a[:5]}..{len(bad_a)}; "
              f"b max {db.max().item():.3g} rows {bad_b[:5]}..{len(bad_b)}", flush=True)
