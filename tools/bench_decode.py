"""Decode throughput: AutoEncoder.decode of B sampled futures for ph frames (config-2 shape:
64 sequences x 50 futures = 3,200 rows, ph = 120), HIP decoder vs the float64 CPU oracle on a
bounded sample.  Prints one JSON line."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import oracle as O  # noqa: E402  (the CPU baseline leg only)
from skeletondiffusion_amd import synthetic  # noqa: E402
from skeletondiffusion_amd.core.network.autoencoder import AutoEncoder  # noqa: E402
from skeletondiffusion_amd.skeletons import skeleton  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 3200
PH = int(sys.argv[2]) if len(sys.argv) > 2 else 120
cuda = torch.device("cuda:0")
_, _, _, types = skeleton("h36m16")
m = AutoEncoder(node_types=torch.from_numpy(types), num_nodes=16, encoder_hidden_size=96, decoder_hidden_size=96,
                latent_size=96, input_size=3, z_activation="tanh", enc_num_layers=1, output_size=3,
                recurrent_arch_enc="StaticGraphGRU", recurrent_arch_decoder="StaticGraphGRU",
                if_consider_hip=False).eval()
synthetic.fill_module_(m, 4321)
m = m.to(cuda)
x2 = (torch.randn(B, 2, 16, 3) * 0.3).to(cuda)
h = (torch.rand(B, 16, 96) * 2 - 1).to(cuda)
m.decode(x2, h, None, ph=PH)
torch.cuda.synchronize()
t0 = time.perf_counter()
reps = 5
for _ in range(reps):
    m.decode(x2, h, None, ph=PH)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / reps
sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
nc = 64
torch.set_num_threads(16)
t0 = time.perf_counter()
O.gru_decode(sd, types, x2[:nc].cpu(), h[:nc].cpu(), PH)
dc = time.perf_counter() - t0
print(json.dumps({"metric": "decoded futures/s (ph frames each)", "rows": B, "ph": PH, "ms_per_decode": dt * 1e3,
                  "value": B / dt, "cpu_oracle_float64": {"rows": nc, "threads": 16, "value": nc / dc}}))
