"""End-to-end evaluation pipeline on one MI355X (the reference's get_prediction,
eval_prepare_model.py:89-121): past embedding (HIP encoder) -> sample() of 50 futures per
sequence (HIP sampler, release Denoiser) -> decode to 120 frames (HIP decoder) -> APD / ADE / FDE
(HIP metrics), on synthetic weights and data of the AMASS shape (J = 21, 30 observed frames,
T = 10 as the release config).  Prints one JSON line with per-stage times and end-to-end futures/s,
next to the reference's published end-to-end rate (12,726 AMASS test segments x 50
futures in ~12 min on an RTX6000 ~ 884 futures/s; data loading included there).

Usage: python tools/eval_pipeline.py [sequences] [T]"""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from bench import build_config  # noqa: E402
from skeletondiffusion_amd import metrics, synthetic  # noqa: E402
from skeletondiffusion_amd.core.network.autoencoder import AutoEncoder  # noqa: E402
from skeletondiffusion_amd.skeletons import skeleton  # noqa: E402

NSEQ = int(sys.argv[1]) if len(sys.argv) > 1 else 256
T = int(sys.argv[2]) if len(sys.argv) > 2 else 10
FUT, OBS, PH = 50, 30, 120
cuda = torch.device("cuda:0")
d, _, _ = build_config("amass21", cuda, T=T, batch=1, futures=FUT)
_, _, _, types = skeleton("amass21")
J = len(types)
ae = AutoEncoder(node_types=torch.from_numpy(types), num_nodes=J, encoder_hidden_size=96, decoder_hidden_size=96,
                 latent_size=96, input_size=3, z_activation="tanh", enc_num_layers=1, output_size=3,
                 recurrent_arch_enc="StaticGraphGRU", recurrent_arch_decoder="StaticGraphGRU",
                 if_consider_hip=False).eval()
synthetic.fill_module_(ae, 4321)
ae = ae.to(cuda)
obs = (torch.from_numpy(synthetic.normal((NSEQ, OBS, J, 3), seed=51)) * 0.3).to(cuda)
target = (torch.from_numpy(synthetic.normal((NSEQ, PH, J, 3), seed=52)) * 0.3).to(cuda)


def run():
    st = {}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
    ev[0].record()
    z_past = ae.get_past_embedding(obs)
    ev[1].record()
    lat, _ = d.sample(batch_size=NSEQ * FUT, x_cond=z_past, seed=7)
    ev[2].record()
    pred = ae.decode(obs.repeat_interleave(FUT, 0), lat, z_past.repeat_interleave(FUT, 0), ph=PH)
    ev[3].record()
    p = pred.view(NSEQ, FUT, PH, J, 3)
    apd = metrics.apd(p)
    ade = metrics.ade(target, p)
    fde = metrics.fde(target, p)
    ev[4].record()
    torch.cuda.synchronize()
    for k, (a, b) in zip(("encode", "sample", "decode", "metrics"), zip(ev, ev[1:])):
        st[k] = a.elapsed_time(b)
    return st, float(apd.mean()), float(ade.mean()), float(fde.mean())


run()  # warm-up: plans, graphs, workspaces
t0 = time.perf_counter()
st, apd, ade, fde = run()
wall = time.perf_counter() - t0
rows = NSEQ * FUT
print(json.dumps({"metric": "end-to-end evaluated futures/s (encode + sample + decode + APD/ADE/FDE)",
                  "value": rows / wall, "unit": "futures/s", "sequences": NSEQ, "futures": FUT, "J": J, "T": T,
                  "obs_frames": OBS, "pred_frames": PH, "wall_ms": wall * 1e3, "stage_ms": st,
                  "apd": apd, "ade": ade, "fde": fde, "data": "synthetic weights and motions",
                  "reference_published": {"value": 884, "unit": "futures/s end-to-end",
                                          "hardware": "NVIDIA RTX6000", "source": "BASELINE.md (README.md:223)"}}))
