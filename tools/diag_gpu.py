"""GPU diagnostics (run on the box): U/eigh reproducibility across machines, graph vs eager."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from conftest import build_release_diffusion, golden, release_inputs  # noqa: E402
from skeletondiffusion_amd.core.diffusion import get_cov_from_corr  # noqa: E402

dev = torch.device("cuda:0")
for key in ["h36m16", "amass21", "freeman17", "mano51"]:
    z = golden("cov_" + key)
    try:
        S, L, U = get_cov_from_corr(torch.from_numpy(z["corr"]))
        print(key, "U maxdiff vs build-container fixture:", float(np.abs(U.numpy() - z["U"]).max()),
              "Lambda maxdiff", float(np.abs(L.numpy() - z["Lambda_N"]).max()),
              "col sign flips", int((np.sign((U.numpy() * z["U"]).sum(0)) < 0).sum()))
    except AssertionError as e:
        print(key, "get_cov_from_corr raised", e)

z = golden("release_h36m16_T10")
d = build_release_diffusion(z, dev)
xc = release_inputs(z)[0].to(dev)
xcs, fu, start, samp = release_inputs(z)
e = d.engine
a = e.sample_loop(8, x_cond=xc, seed=77, graph=False)[0].clone()
b = e.sample_loop(8, x_cond=xc, seed=77, graph=True)[0].clone()
print("device noise graph vs eager:", float((a - b).abs().max()))
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    b2 = e.sample_loop(8, x_cond=xc, seed=77, graph=True)[0].clone()
    a2 = e.sample_loop(8, x_cond=xc, seed=77, graph=False)[0].clone()
torch.cuda.synchronize()
print("on side stream: graph vs eager:", float((a2 - b2).abs().max()), " eager(default) vs eager(side):",
      float((a - a2).abs().max()))
st, sn = start.to(dev), samp.to(dev)
h1 = e.sample_loop(8, x_cond=xc, start_noise=st, sampling_noise=sn, graph=False)[0].clone()
h2 = e.sample_loop(8, x_cond=xc, start_noise=st, sampling_noise=sn, graph=True)[0].clone()
torch.cuda.synchronize()
print("host noise graph vs eager:", float((h1 - h2).abs().max()))
