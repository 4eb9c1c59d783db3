"""Half precision mode (reduced-precision activations, quality gate
"latent ADE and APD within 1 % of the fp32 path").  Mode "half" runs the graph-linear launches
on one f16 product per multiply-add (f32 accumulate, f32 activations in HBM); the gate is
measured here on the sampler's own outputs with the on-device metrics (the reference's
multimodal.py formulas), against the f32-accurate mode on identical inputs and noise."""
import pytest
import torch

from conftest import build_release_diffusion, golden
from skeletondiffusion_amd import _lib, metrics
from skeletondiffusion_amd._lib import SkelDiffError

pytestmark = pytest.mark.gpu


def _gate(name, cuda, T):
    z = golden(name)
    d = build_release_diffusion(z, cuda, T=T)
    J = z["corr"].shape[0]
    nseq, S = 16, 50  # 800 rows, 50 futures per sequence as in the evaluation (eval_prepare_model.py:96)
    g = torch.Generator().manual_seed(7)
    xc = (torch.rand((nseq, J, 96), generator=g) * 2 - 1).to(cuda)
    target = (torch.rand((nseq, J, 96), generator=g) * 2 - 1).to(cuda)  # fixed synthetic target
    eng = d.engine
    out = {}
    for prec in ("f32", "half", "f32"):
        eng.set_precision(prec)
        img = eng.sample_loop(nseq * S, x_cond=xc, seed=5)[0].clone()
        lat = img.view(nseq, S, J, 96)
        out.setdefault(prec, []).append((img, metrics.lat_apd(lat), metrics.apd(lat.view(nseq, S, 1, J * 96)),
                                         metrics.ade(target.view(nseq, 1, J * 96), lat.view(nseq, S, 1, J * 96))))
    eng.set_precision("f32")
    torch.cuda.synchronize()
    (f_img, f_lapd, f_apd, f_ade), (f2_img, *_) = out["f32"]
    h_img, h_lapd, h_apd, h_ade = out["half"][0]
    assert torch.equal(f_img, f2_img)          # switching back restores the f32 launches bitwise
    assert not torch.equal(f_img, h_img)       # and the half launches really ran
    diff = (h_img - f_img).abs().max().item()
    for a, b in ((h_lapd, f_lapd), (h_apd, f_apd), (h_ade, f_ade)):
        rel = abs(a.mean().item() - b.mean().item()) / b.mean().item()
        assert rel < 0.01, (name, rel)
    return diff


@pytest.mark.parametrize("name,T", [("release_freeman17_T10", 10), ("release_h36m16_T10", 10),
                                    ("release_amass21_T10", 10)])
def test_half_precision_quality_gate(name, T, cuda):
    diff = _gate(name, cuda, T)
    assert diff < 0.1  # per-latent drift stays small (the latents are O(1))


def test_precision_mode_validation(cuda):
    z = golden("release_h36m16_T10")
    d = build_release_diffusion(z, cuda)
    with pytest.raises(SkelDiffError):
        d.engine.set_precision("bf8")
    assert _lib.lib().sd_plan_set_precision(d.engine.plan(), 2) < 0
    assert d.engine.precision == "f32"
