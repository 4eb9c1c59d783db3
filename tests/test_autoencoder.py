"""Graph-GRU autoencoder against the reference's own AutoEncoder outputs
(tests/golden/decoder.npz, gen_golden.py:gen_decoder): the oracle restatement and the mirrored
modules on CPU, the HIP decoder (sd_gru_decode) on the GPU.  Tolerance 1e-4 on the decoded
frames (fp32; 120 recurrent steps)."""
import numpy as np
import pytest
import torch

import oracle as O
from conftest import golden
from skeletondiffusion_amd import synthetic
from skeletondiffusion_amd.skeletons import skeleton

AE_KW = dict(num_nodes=16, encoder_hidden_size=96, decoder_hidden_size=96, latent_size=96, input_size=3,
             z_activation="tanh", enc_num_layers=1, output_size=3, recurrent_arch_enc="StaticGraphGRU",
             recurrent_arch_decoder="StaticGraphGRU", if_consider_hip=False)
TOL = 1e-4


def _model(device="cpu"):
    from skeletondiffusion_amd.core.network.autoencoder import AutoEncoder

    _, _, _, types = skeleton("h36m16")
    m = AutoEncoder(node_types=torch.from_numpy(types), **AE_KW).eval()
    synthetic.fill_module_(m, 4321)
    return m.to(device), types


def _inputs():
    past = torch.from_numpy(synthetic.normal((3, 30, 16, 3), seed=41)) * 0.3
    lat = torch.from_numpy(synthetic.uniform((12, 16, 96), seed=42))
    return past, lat


def test_state_dict_keys_match_reference():
    m, _ = _model()
    assert sorted(m.state_dict().keys()) == list(golden("decoder")["keys"])


def test_oracle_matches_reference():
    z = golden("decoder")
    m, types = _model()
    sd = {k: v.detach() for k, v in m.state_dict().items()}
    past, lat = _inputs()
    out = O.gru_decode(sd, types, past.repeat_interleave(4, 0)[:, -2:], lat, 120)
    assert (out - torch.from_numpy(z["out"])).abs().max().item() < 1e-5
    zp = O.gru_encode(sd, types, past)
    assert (zp - torch.from_numpy(z["z_past"])).abs().max().item() < 1e-5


def test_module_torch_paths_match_reference():
    """Encoder (past embedding) and the training-time torch Decoder.forward."""
    z = golden("decoder")
    m, _ = _model()
    past, lat = _inputs()
    with torch.no_grad():
        zp = m.z_activation(m(past))  # the torch encoder (training path)
        out, _ = m.decoder(x=past.repeat_interleave(4, 0)[:, -2:], h=lat, z=None, ph=120)
    assert (zp - torch.from_numpy(z["z_past"])).abs().max().item() < 1e-5
    assert (out - torch.from_numpy(z["out"])).abs().max().item() < 1e-5


def test_decode_and_encode_refuse_cpu():
    from skeletondiffusion_amd._lib import SkelDiffError

    m, _ = _model()
    past, lat = _inputs()
    with pytest.raises(SkelDiffError):
        m.decode(past[:1], lat[:1], None, ph=3)
    with pytest.raises(SkelDiffError):
        m.get_past_embedding(past[:1])


@pytest.mark.gpu
def test_hip_encode_matches_reference(cuda):
    z = golden("decoder")
    m, types = _model(cuda)
    past, _ = _inputs()
    zp = m.get_past_embedding(past.to(cuda))
    torch.cuda.synchronize()
    assert (zp.cpu() - torch.from_numpy(z["z_past"])).abs().max().item() < TOL
    g = torch.Generator().manual_seed(5)
    x = torch.randn((7, 9, 16, 3), generator=g) * 0.3  # ragged batch, other length
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    ref = O.gru_encode(sd, types, x)
    got = m.get_past_embedding(x.to(cuda))
    torch.cuda.synchronize()
    assert (got.cpu() - ref).abs().max().item() < TOL


@pytest.mark.gpu
def test_hip_decode_matches_reference(cuda):
    z = golden("decoder")
    m, _ = _model(cuda)
    past, lat = _inputs()
    out = m.decode(past.repeat_interleave(4, 0).to(cuda), lat.to(cuda), None, ph=120)
    torch.cuda.synchronize()
    assert out.shape == (12, 120, 16, 3)
    assert (out.cpu() - torch.from_numpy(z["out"])).abs().max().item() < TOL


@pytest.mark.gpu
@pytest.mark.parametrize("B,ph", [(1, 5), (37, 30), (0, 4)])
def test_hip_decode_matches_oracle_ragged(B, ph, cuda):
    m, types = _model(cuda)
    g = torch.Generator().manual_seed(B)
    x2 = torch.randn((B, 2, 16, 3), generator=g) * 0.3
    h = torch.rand((B, 16, 96), generator=g) * 2 - 1
    out = m.decode(x2.to(cuda), h.to(cuda), None, ph=ph)
    torch.cuda.synchronize()
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    ref = O.gru_decode(sd, types, x2, h, ph)
    assert out.shape == (B, ph, 16, 3)
    if B:
        assert (out.cpu() - ref).abs().max().item() < TOL
