"""Per-shape microbenchmark of the graph-linear kernel (through the ABI test hook) on the
release Denoiser's layer shapes at B rows, J=16, 10 node types.  Prints TFLOP/s per shape.
Variants are chosen by env vars read once per process (SKELDIFF_GL_VARIANT, SKELDIFF_GL_NCB)."""
import ctypes
import os
import sys

os.environ.setdefault("SKELDIFF_GL_CACHE_SPLIT", "1")  # split weights once, not per timed call
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from skeletondiffusion_amd import _lib  # noqa: E402

B = int(os.environ.get("ROWS", "3200"))
J, NT = 16, 10
dev = torch.device("cuda:0")
L = _lib.lib()
types = (ctypes.c_int64 * J)(*[0, 1, 2, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 7, 8, 9])
SHAPES = [  # name, K1, K2, N, bias, film, act, res, rms, per-step count
    ("init_lin", 96, 96, 192, 1, 0, 0, 0, 0, 1), ("res_block1", 192, 0, 192, 1, 1, 1, 0, 0, 8),
    ("res_block2", 192, 0, 192, 1, 0, 1, 1, 0, 8), ("to_qkv", 192, 0, 768, 0, 0, 0, 0, 1, 7),
    ("to_out", 256, 0, 192, 0, 0, 0, 1, 0, 7), ("final_b1/res", 192, 192, 192, 1, 1, 1, 0, 0, 2),
    ("final_b2", 192, 0, 192, 1, 0, 1, 1, 0, 1), ("final_glin", 192, 0, 96, 1, 0, 0, 0, 0, 1)]
tag = f"v{os.environ.get('SKELDIFF_GL_VARIANT', '0')}/t{os.environ.get('SKELDIFF_GL4_CFG', 'auto')}"
tot_f = tot_t = 0.0
only = os.environ.get("SHAPE")
for name, K1, K2, N, bias, film, act, res, rms, cnt in SHAPES:
    if only and name != only:
        continue
    g = torch.Generator(dev).manual_seed(0)
    x1 = torch.randn(B, J, K1, device=dev, generator=g)
    x2 = torch.randn(B, J, K2, device=dev, generator=g) if K2 else None
    W = torch.randn(NT, N, K1 + K2, device=dev, generator=g) * 0.05
    bb = torch.randn(NT, N, device=dev, generator=g) if bias else None
    fl = torch.randn(2 * N, device=dev, generator=g) if film else None
    rr = torch.randn(B, J, N, device=dev, generator=g) if res else None
    gh = torch.softmax(torch.randn(J, J, device=dev, generator=g), -1)
    out = torch.empty(B, J, N, device=dev)
    p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    call = lambda: L.sd_test_graph_linear(p(x1), K1, 1, p(x2), K2, p(W), p(bb), types, p(gh), p(fl), act, p(rr),  # noqa: E731
                                          p(out), B, J, N, rms, 0)
    for _ in range(3):
        _lib.check(call())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record()
    for _ in range(reps):
        call()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    flops = 2.0 * B * J * N * (K1 + K2) + 2.0 * B * J * J * N
    tot_f += flops * cnt
    tot_t += ms * cnt
    print(f"{tag:12s} {name:14s} K={K1 + K2:4d} N={N:4d}  {ms * 1e3:8.1f} us  {flops / ms / 1e9:7.1f} TF/s")
print(f"{tag:12s} per-step graph-linear: {tot_t:.3f} ms  {tot_f / tot_t / 1e9:.1f} TF/s")
