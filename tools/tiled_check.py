"""GPU check of the tiled split route (k_gl4t + k_gl4 MODE 2 / 3, split_route option 3): the
whole sampler at the config-2 shape must be bitwise equal to the one-kernel route.
usage: python tools/tiled_check.py [config] [T] [sequences]"""
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import bench  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "amass16"
T = int(sys.argv[2]) if len(sys.argv) > 2 else 4
nseq = int(sys.argv[3]) if len(sys.argv) > 3 else 64
dev = torch.device("cuda", 0)
d, xc, rows = bench.build_config(cfg, dev, T=T, batch=nseq)
eng = d.engine
J, D = d.channels, d.seq_length
res = {}
RUNS = [("one-kernel", dict(split_route=1, row_chains=3)), ("tiled 1 chain", dict(split_route=3, row_chains=1)),
        ("tiled 3 chains", dict(split_route=3, row_chains=3)), ("tiled 2 chains", dict(split_route=3, row_chains=2)),
        ("one-kernel 1 chain", dict(split_route=1, row_chains=1))]
if os.environ.get("TILED_RUNS"):
    RUNS = [r for r in RUNS if r[0] in os.environ["TILED_RUNS"].split(",")] 
for name, opts in RUNS:
    for k, v in opts.items():
        eng.set_option(k, v)
    out = torch.empty((rows, J, D), device=dev)
    for graph in (False, True):
        eng.sample_loop(rows, x_cond=xc, seed=77, row0=0, graph=graph, out=out, keep_start=False)
        torch.cuda.synchronize()
        st = eng.status(rows)
        if st:
            print(f"{name} graph={graph}: workspace status word {st:#x}")
        res[(name, graph)] = out.clone()
ref = res[("one-kernel", False)]
ok = True
for k, v in res.items():
    diff = (v - ref).abs().max().item()
    nbad = int((v != ref).sum().item())
    rows_bad = ((v != ref).flatten(1).any(1)).nonzero().flatten().tolist()
    per = [sum(1 for r in rows_bad if a <= r < b) for a, b in ((0, 1056), (1056, 2112), (2112, rows))]
    print(f"{k[0]:>20s} graph={k[1]!s:5s} max|d|={diff:.3e} differing={nbad} rows by chain={per}"
          + (f" first rows {rows_bad[:12]}" if rows_bad else ""))
    ok = ok and nbad == 0
print("BITWISE OK" if ok else "BITWISE MISMATCH")
sys.exit(0 if ok else 1)
