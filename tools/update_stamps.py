"""Timeline of one full-batch update launch (k_update_mfma<16, 4, 6>: config 2's 3,200 rows, one row
chain, T = 10, eager) from the diagnostic build's in-kernel stamps (SD_UPD_STAMPS):
per workgroup, thread 0's s_memrealtime (100 MHz) at entry, loads issued, phase A done, barrier,
x0 fragments in use, MFMAs done, stores acknowledged, and its CU.
usage (GPU box): SKELDIFF_LIB=$PWD/skeletondiffusion_amd/libskeldiff_ustamps.so python tools/update_stamps.py"""
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
eng.set_option("row_chains", 1)
fn = _lib.lib().sd_debug_update_stamps
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
nwg = (rows + 3) // 4
buf = np.zeros((nwg, 8), dtype=np.uint64)
names = ["loads issued", "phase A", "barrier", "x0 arrived", "MFMAs", "stores acked"]
for rep in range(3):
    assert fn(None, 0, 1) == 0
    eng.sample_loop(rows, x_cond=xc, seed=rep, graph=False)
    torch.cuda.synchronize()
    assert fn(buf.ctypes.data, nwg, 0) == 0
    t = buf[:, :7].astype(np.int64)
    base = t[:, 0].min()
    rel = (t - base) * 10 / 1e3  # us from the first workgroup's entry
    print(f"rep {rep}: {nwg} workgroups on {len(set(buf[:, 7].tolist()))} CUs, launch span {rel[:, 6].max():.1f} us")
    print(f"  entry           min {rel[:, 0].min():5.2f}  median {np.median(rel[:, 0]):5.2f}  max {rel[:, 0].max():5.2f} us")
    for k, n in enumerate(names, start=1):
        dur = (t[:, k] - t[:, k - 1]) * 10 / 1e3
        print(f"  {n:15s} at median {np.median(rel[:, k]):5.2f} (max {rel[:, k].max():5.2f}) us;"
              f"  phase median {np.median(dur):5.2f}  p90 {np.percentile(dur, 90):5.2f} us")
