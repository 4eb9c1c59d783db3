"""Route / row-chain sweep on one GPU (DESIGN.md §4c, §4d''): for each BASELINE config shape,
futures/s of the whole sampler (hipGraph, device noise, reused output buffer -- bench.py's timed
call) under each (split_route, row_chains) pair, in one process.  Same-box A/B: the plan defaults
are chosen from these numbers.
usage: python tools/sweep_routes.py [config[:batch][:T] ...]   (default: the bench shapes)"""
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import bench  # noqa: E402

DEFAULT = ["amass16", "amass16:32", "amass16:16", "amass16:8", "freeman17", "amass21", "mano51", "h36m_t1000",
           "freeman17_bf16:1377:10"]
ROUTES = {"amass16": [0, 1, 2, 3], "amass21": [0, 2, 3], "freeman17": [0, 2, 3],
          "freeman17_bf16": [0, 1, 3], "mano51": [0], "h36m_t1000": [0, 1, 2, 5]}
ROUTES = {k: [int(x) for x in os.environ["SWEEP_ROUTES"].split(",")] for k in ROUTES} if os.environ.get("SWEEP_ROUTES") \
    else ROUTES
CHAINS = [int(x) for x in os.environ.get("SWEEP_CHAINS", "1,2,3").split(",")]
dev = torch.device("cuda", 0)
out_rows = []
for spec in (sys.argv[1:] or DEFAULT):
    parts = spec.split(":")
    cfg = parts[0]
    batch = int(parts[1]) if len(parts) > 1 else None
    T = int(parts[2]) if len(parts) > 2 else None
    d, xc, rows = bench.build_config(cfg, dev, T=T, batch=batch)
    c = bench.CONFIGS[cfg]
    eng = d.engine
    eng.set_precision(c.get("precision", "f32"))
    out = torch.empty((rows, d.channels, d.seq_length), device=dev)
    steps = 2 if d.num_timesteps >= 1000 else 5
    for route in ROUTES.get(cfg.split("_")[0] if cfg not in ROUTES else cfg, [0]):
        for n in CHAINS:
            if (rows + 31) // 32 < n and n > 1:
                continue
            eng.set_option("split_route", route)
            eng.set_option("row_chains", n)
            try:
                for i in range(2):
                    eng.sample_loop(rows, x_cond=xc, seed=100 + i, graph=True, out=out, keep_start=False)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(steps):
                    eng.sample_loop(rows, x_cond=xc, seed=i, graph=True, out=out, keep_start=False)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / steps
            except Exception as e:  # a route that does not apply to the shape
                print(f"{spec} route {route} chains {n}: {e}", flush=True)
                continue
            r = {"config": spec, "rows": rows, "T": d.num_timesteps, "split_route": route, "row_chains": n,
                 "ran_chains": eng.get_option("last_chains"), "futures_per_s": rows / dt, "ms": dt * 1e3}
            out_rows.append(r)
            print(json.dumps(r), flush=True)
    del d, eng, out
    torch.cuda.empty_cache()
best = {}
for r in out_rows:
    k = r["config"]
    if k not in best or r["futures_per_s"] > best[k]["futures_per_s"]:
        best[k] = r
print("BEST", json.dumps(best))
