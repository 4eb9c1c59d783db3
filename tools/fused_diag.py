"""Diagnostic: the fused layer route (split_route 6) vs the tiled split route (3) -- final latents
and every recorded step, with cross-step matches (is a record shifted?).  GPU only.
usage: python tools/fused_diag.py [batch] [T] [chains]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import build_config  # noqa: E402


def main():
    batch, T, chains = (int(a) for a in (sys.argv[1:] + ["64", "4", "1"][len(sys.argv) - 1:])[:3])
    cuda = torch.device("cuda:0")
    d, x_cond, rows = build_config("amass16", cuda, T=T, batch=batch)
    eng = d.engine
    eng.set_option("row_chains", chains)
    runs = {}
    for route in (3, 3, 6, 6):
        eng.set_option("split_route", route)
        for rec in ((False, True), (True, False)):
            r = eng.sample_loop(rows, x_cond=x_cond, seed=31, record=rec, graph=False)
            torch.cuda.synchronize()
            runs.setdefault((route, rec), []).append([None if t is None else t.clone() for t in r])
        print("route", route, "last_route", eng.get_option("last_route"), "status", eng.status(rows))
    names = ("img", "start", "noise_t", "mean_t", "imgs")
    for rec in ((False, True), (True, False)):
        a3, b3 = runs[(3, rec)]
        a6, b6 = runs[(6, rec)]
        for i, n in enumerate(names):
            if a3[i] is None:
                continue
            e = lambda x, y: float((x - y).abs().max())  # noqa: E731
            print(rec, n, "3 vs 3", e(a3[i], b3[i]), "6 vs 6", e(a6[i], b6[i]), "3 vs 6", e(a3[i], a6[i]))
            if a3[i].dim() == 4:
                for k in range(a3[i].shape[1]):
                    per = [e(a3[i][:, k], a6[i][:, kk]) for kk in range(a3[i].shape[1])]
                    rows_bad = int(((a3[i][:, k] - a6[i][:, k]).abs().amax(dim=(1, 2)) > 0).sum())
                    print(f"   step {k}: vs 6's steps {['%.2e' % v for v in per]}  rows differing {rows_bad}/{rows}")


if __name__ == "__main__":
    main()
