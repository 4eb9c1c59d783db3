"""Timeline of one k_gl4t launch (N = 192, K = 192, config 2's full batch, one row chain) from the
diagnostic build's in-kernel stamps (SD_GL4T_STAMPS): per workgroup the entry, the
end of the K loop and the end of its Y stores (s_memrealtime, 100 MHz), and its CU.
usage (GPU box): SKELDIFF_LIB=$PWD/skeletondiffusion_amd/libskeldiff_stamps.so python tools/gl4t_stamps.py"""
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import bench  # noqa: E402
from skeletondiffusion_amd import _lib  # noqa: E402

dev = torch.device("cuda", 0)
d, xc, rows = bench.build_config("amass16", dev, T=10)
eng = d.engine
L = _lib.lib()
fn = L.sd_debug_gl4t_stamps
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
x = torch.randn(rows, d.channels, d.seq_length, device=dev)
xcr = xc.repeat_interleave(rows // xc.shape[0], 0)
for _ in range(3):
    eng.denoiser_forward(x, 5, x_cond=xcr)
torch.cuda.synchronize()
nwg = int(os.environ.get("NWG", 25 * 16))
buf = np.zeros((nwg, 4), dtype=np.uint64)
for rep in range(3):
    assert fn(None, 0, 1) == 0
    eng.denoiser_forward(x, 5, x_cond=xcr)
    torch.cuda.synchronize()
    assert fn(buf.ctypes.data, nwg, 0) == 0
    t0, t1, t2, cu = (buf[:, i].astype(np.int64) for i in range(4))
    base = t0.min()
    s, k, e = (t0 - base) * 10, (t1 - base) * 10, (t2 - base) * 10  # ns
    print(f"rep {rep}: {nwg} workgroups, launch span {(e.max()) / 1e3:.1f} us")
    print(f"  entry: min 0 / median {np.median(s) / 1e3:.2f} / max {s.max() / 1e3:.2f} us")
    print(f"  K loop (entry -> loop end): median {np.median(k - s) / 1e3:.2f} us, min {np.min(k - s) / 1e3:.2f}, max {np.max(k - s) / 1e3:.2f}")
    print(f"  stores (loop end -> last store acked): median {np.median(e - k) / 1e3:.2f} us, max {np.max(e - k) / 1e3:.2f}")
    print(f"  loop end: median {np.median(k) / 1e3:.2f} / max {k.max() / 1e3:.2f} us; store end: median {np.median(e) / 1e3:.2f} us")
    print(f"  distinct CUs {len(np.unique(cu))}; workgroups per CU max {np.bincount(cu.astype(np.int64)).max()}")
    ckb = np.zeros((nwg, 2), dtype=np.uint64)
    fk = L.sd_debug_gl4t_clock
    fk.restype = ctypes.c_int
    fk.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert fk(ckb.ctypes.data, nwg) == 0
    cyc = ckb[:, 1].astype(np.int64) - ckb[:, 0].astype(np.int64)
    ghz = cyc / np.maximum(k - s, 1)  # shader cycles per ns over the K loop
    print(f"  shader clock over the K loop: median {np.median(ghz):.2f} GHz; K-loop cycles median {np.median(cyc):.0f} "
          f"({np.median(cyc) / 12:.0f} per 16-deep chunk; 18 MFMAs = 576 issue cycles)")
    hist = np.histogram(k / 1e3, bins=8)
    print("  loop-end histogram (us):", [f"{b:.1f}:{c}" for b, c in zip(hist[1][:-1], hist[0])])
    if os.environ.get("SKELDIFF_GL4T_CFG", "0") in ("0", "1"):  # per-chunk barrier stamps (staged forms)
        ch = np.zeros((nwg, 16), dtype=np.uint64)
        fc = L.sd_debug_gl4t_chunk_stamps
        fc.restype = ctypes.c_int
        fc.argtypes = [ctypes.c_void_p, ctypes.c_int]
        assert fc(ch.ctypes.data, nwg) == 0
        c = (ch[:, :12].astype(np.int64) - base) * 10  # ns after the launch's first entry
        print("  chunk barrier passed (median over workgroups, us):", " ".join(f"{np.median(c[:, i]) / 1e3:.2f}" for i in range(12)))
        print("  per-chunk gaps (median, us):", " ".join(f"{np.median(c[:, i + 1] - c[:, i]) / 1e3:.2f}" for i in range(11)))
