"""§4c hazard bisection with the diagnostic library (libskeldiff_dbg.so, -DSD_DEBUG_LDS).

Runs the config-2 sampler (J=16, B=3200) with 1 row chain (reference) and then 3 / 2 chains,
eager and graph, with the plan's v4 weight staging set to `staging` (0 LDS-DMA + whole-CU LDS,
the default; 1 register-staged; 2 the diagnostic LDS-DMA-with-shared-CU mode that reproduces the
corruption), and prints per run: max |diff| vs the 1-chain result, the number of differing rows
and, with the diagnostic library, the LDS integrity counters ([0] k_gl4 weight stages vs global,
[1] k_update tables vs global, [2] k_gl4 G-hat table).  Usage (GPU box):
    python tools/lds_hazard.py [T] [staging]
    SKELDIFF_LIB=skeletondiffusion_amd/libskeldiff_dbg.so python tools/lds_hazard.py 20 2
(build the diagnostic library with `python -m skeletondiffusion_amd.build --debug-lds`)
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, ".")
from bench import build_config  # noqa: E402
from skeletondiffusion_amd import _lib  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 20
staging = int(sys.argv[2]) if len(sys.argv) > 2 else 2
cuda = torch.device("cuda:0")
d, x_cond, rows = build_config("amass16", cuda, T=T)
d.engine.set_option("gl4_staging", staging)
L = _lib.lib()
dbg = (ctypes.c_uint32 * 8)()
has_dbg = hasattr(L, "sd_debug_lds_counters")


def counters():
    if not has_dbg:
        return None
    _lib.check(L.sd_debug_lds_counters(dbg))
    return list(dbg)[:3]


d.engine.set_option("row_chains", 1)
ref = d.engine.sample_loop(rows, x_cond=x_cond, seed=11, graph=False)[0].clone()
torch.cuda.synchronize()
print(f"lib={_lib.LIB_PATH} staging={staging} T={T} 1 chain: counters {counters()}",
      flush=True)
for graph in (False, True):
    for n in (3, 3, 2):
        d.engine.set_option("row_chains", n)
        a = d.engine.sample_loop(rows, x_cond=x_cond, seed=11, graph=graph)[0].clone()
        torch.cuda.synchronize()
        da = (a - ref).abs().view(rows, -1).amax(1)
        bad = torch.nonzero(da).flatten().tolist()
        print(f"graph={graph} chains={n}: max {da.max().item():.3g}, {len(bad)} rows differ "
              f"(first {bad[:4]}); counters {counters()}", flush=True)
