"""Run-to-run determinism of sample_loop under the current process defaults (SKELDIFF_*):
repeat the same seeded chain and print max |diff| to the first run."""
import sys

import torch

sys.path.insert(0, ".")
from bench import build_config  # noqa: E402

cfg, batch, T, reps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
chains = int(sys.argv[5]) if len(sys.argv) > 5 else 3
dev = torch.device("cuda:0")
d, x_cond, rows = build_config(cfg, dev, T=T, batch=batch)
eng = d.engine
eng.set_option("row_chains", chains)
ref = None
for graph in (False, True):
    for r in range(reps):
        x = eng.sample_loop(rows, x_cond=x_cond, seed=5, graph=graph)[0].clone()
        torch.cuda.synchronize()
        if ref is None:
            ref = x
        diff = (x - ref).abs()
        print(cfg, rows, "T", T, "chains", chains, "graph", graph, "rep", r, "max", float(diff.max()),
              "nbad", int((diff > 0).sum()), "status", eng.status(rows), flush=True)
        bad_rows = torch.nonzero(diff.flatten(1).amax(1) > 0).flatten().tolist()
        if bad_rows:
            print("   rows", len(bad_rows), bad_rows[:12], "...", bad_rows[-6:], flush=True)
