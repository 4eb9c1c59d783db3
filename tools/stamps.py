"""Phase timing of one graph-linear launch from in-kernel s_memrealtime stamps (v4, SKELDIFF_GL4_CFG=6):
per workgroup [start, first chunk done, K loop done, scaled, epilogue done, final barrier] -> µs
percentiles across workgroups relative to the earliest start."""
import ctypes
import os
import sys

os.environ.setdefault("SKELDIFF_GL_CACHE_SPLIT", "1")
import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from skeletondiffusion_amd import _lib  # noqa: E402

L = _lib.lib()
dev = torch.device("cuda:0")
B, J, NT = int(os.environ.get("ROWS", "3200")), 16, 10
types = (ctypes.c_int64 * J)(*[0, 1, 2, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 7, 8, 9])
K, N = int(os.environ.get("K", "192")), int(os.environ.get("N", "192"))
res = os.environ.get("RES", "0") == "1"
g = torch.Generator(dev).manual_seed(0)
x1 = torch.randn(B, J, K, device=dev, generator=g)
W = torch.randn(NT, N, K, device=dev, generator=g) * 0.05
bb = torch.randn(NT, N, device=dev, generator=g)
fl = torch.randn(2 * N, device=dev, generator=g)
rr = torch.randn(B, J, N, device=dev, generator=g) if res else None
gh = torch.softmax(torch.randn(J, J, device=dev, generator=g), -1)
out = torch.empty(B, J, N, device=dev)
p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
for it in range(5):
    _lib.check(L.sd_test_graph_linear(p(x1), K, 1, None, 0, p(W), p(bb), types, p(gh), p(fl), 1, p(rr), p(out), B, J,
                                      N, 0, 0))
torch.cuda.synchronize()
nwg = ((N + 95) // 96) * ((B + 31) // 32)  # v4 default J=16 tile: 32 rows x 96 columns
st = out.view(-1)[: nwg * 8].view(torch.int32).cpu().numpy().astype(np.int64).reshape(nwg, 8) & 0xFFFFFFFF
t = (st[:, :6] - st[:, 0].min()) / 100.0  # 100 MHz -> µs
names = ["start", "chunk0+1", "kloop", "scaled", "epilogue", "barrier"]
print(f"K={K} N={N} rows={B} res={res}: {nwg} workgroups, {len(set(st[:, 6]))} distinct CUs(smid)")
kl_us = (st[:, 2] - st[:, 1]) / 100.0
ghz = st[:, 7] / np.maximum(kl_us, 1e-3) / 1e3
print(f"  shader clock over the K loop: median {np.median(ghz):.2f} GHz (min {ghz.min():.2f}, max {ghz.max():.2f})")
for i, n in enumerate(names):
    q = np.percentile(t[:, i], [0, 50, 100])
    print(f"  {n:9s} min {q[0]:7.2f}  med {q[1]:7.2f}  max {q[2]:7.2f} µs")
d = np.diff(t, axis=1)
for i in range(5):
    q = np.percentile(d[:, i], [0, 50, 100])
    print(f"  {names[i]}->{names[i+1]:9s} min {q[0]:7.2f}  med {q[1]:7.2f}  max {q[2]:7.2f} µs")
cyc = out.view(-1)[nwg * 8: nwg * 8 + nwg * 8 * 4].view(torch.int32).cpu().numpy().astype(np.int64).reshape(nwg * 8, 4)
print("  chunk 5, per wave (shader cycles): median [vmcnt wait, barrier, issue loads, compute]:",
      np.median(cyc, axis=0).astype(int), " p90:", np.percentile(cyc, 90, axis=0).astype(int))

