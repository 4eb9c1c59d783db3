"""The posterior update kernel alone under rocprofv3 --kernel-trace: config 2's 3,200 rows, one
row chain, T = 10, eager, with (a) device Philox noise, (b) given noise (no Philox in the kernel),
(c) the element-per-thread forms (update_kernel 1) -- what each part of k_update_mfma costs.
usage: rocprofv3 --kernel-trace --stats -d <dir> -o run -- python3 tools/update_probe.py <mode> [update_kernel]
(mode: device | given | elementwise; update_kernel: the SD_OPT_UPDATE_KERNEL value, default 0)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import build_config  # noqa: E402


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "device"
    cuda = torch.device("cuda:0")
    d, x_cond, rows = build_config("amass16", cuda, T=10)
    eng = d.engine
    eng.set_option("row_chains", 1)
    if mode == "elementwise":
        eng.set_option("update_kernel", 1)
    elif len(sys.argv) > 2:
        eng.set_option("update_kernel", int(sys.argv[2]))
    J, D = d.channels, d.seq_length
    samp = torch.randn((rows, 9, J, D), device=cuda) if mode == "given" else None
    for _ in range(4):
        eng.sample_loop(rows, x_cond=x_cond, seed=3, sampling_noise=samp, graph=False)
    torch.cuda.synchronize()
    print(mode, "done", eng.get_option("last_route"))


if __name__ == "__main__":
    main()
