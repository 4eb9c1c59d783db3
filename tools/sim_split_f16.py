"""Numerical study (CPU, test infrastructure): what does computing every StaticGraphLinear GEMM as
3 x f16 products (x_hi*W_hi + 2^-11 (x_hi*W_lo + x_lo*W_hi), f32 accumulate) - the scheme of the
v4 graph-linear kernel - do to the sampled latents, next to the exact-f32 oracle and an f64 run?

Usage: python tools/sim_split_f16.py [fixture]   (default release_h36m16_T100)
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle as O  # noqa: E402
from conftest import golden, release_inputs, pinned_cov  # noqa: E402
import oracle.skeldiff_oracle as OS  # noqa: E402

S11 = 2048.0


def split(v):
    hi = v.to(torch.float16)
    lo = ((v - hi.to(v.dtype)) * S11).to(torch.float16)
    return hi.to(torch.float32), lo.to(torch.float32)


def mm_split(x, w):  # x (..., K), w (..., K, N) -> x @ w with f16 split products
    xh, xl = split(x)
    wh, wl = split(w)
    return torch.matmul(xh, wh) + (torch.matmul(xh, wl) + torch.matmul(xl, wh)) / S11


orig_gl = OS._Net.graph_linear
orig_emb = OS.sinusoidal_embedding


def gl_split(self, name, x):
    W = self.w(name + ".weight")
    G = self.w(name + ".G")
    g = torch.nn.functional.normalize(G, p=1.0, dim=1) if self.cfg.learn_influence else G
    if W.dim() == 3:
        w = W[self.types]                      # (J, out, in)
        y = mm_split(x.transpose(0, 1), w.transpose(-2, -1)).transpose(0, 1)
    else:
        y = mm_split(x, W.transpose(-2, -1))
    if self.has(name + ".bias"):
        bias = self.w(name + ".bias")
        y = y + (bias[self.types] if bias.dim() == 2 else bias)
    return g.matmul(y)


def run(fx, mode):
    z = golden(fx)
    J = z["corr"].shape[0]
    cfg = O.release_config(J, z["node_types"])
    sd = O.synthetic_state_dict(cfg, 1234, float(z["final_scale"]))
    S, L, U = pinned_cov(J)
    T = int(z["T"])
    bufs = O.nonisotropic_buffers(S, L, U, O.beta_schedule("cosine", T).double())
    xc, fu, start, samp = release_inputs(z)
    if mode == "f64":
        sd = {k: v.double() for k, v in sd.items()}
        bufs = {k: v.double() for k, v in bufs.items()}
        xc, start, samp = xc.double(), start.double(), samp.double()
    OS._Net.graph_linear = gl_split if mode == "split" else orig_gl
    OS.sinusoidal_embedding = (lambda *a, **k: orig_emb(*a, **k).double()) if mode == "f64" else orig_emb
    img, _ = O.p_sample_loop(sd, cfg, bufs, start, samp, x_cond=xc)
    OS._Net.graph_linear = orig_gl
    OS.sinusoidal_embedding = orig_emb
    return img.double(), torch.from_numpy(z["img"]).double()


if __name__ == "__main__":
    fx = sys.argv[1] if len(sys.argv) > 1 else "release_h36m16_T100"
    f32, ref = run(fx, "f32")
    f64, _ = run(fx, "f64")
    sp, _ = run(fx, "split")
    print(f"{fx}: |f32 - reference| {float((f32 - ref).abs().max()):.3e}")
    print(f"{fx}: |f32 - f64|       {float((f32 - f64).abs().max()):.3e}")
    print(f"{fx}: |split - f64|     {float((sp - f64).abs().max()):.3e}")
    print(f"{fx}: |split - ref|     {float((sp - ref).abs().max()):.3e}  (bar 1e-4)")
