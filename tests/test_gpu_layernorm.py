"""GPU parity of the Denoiser's norm_type='layer' (Block: proj -> LayerNorm over the node axis ->
FiLM -> tanh, reference attention.py:19-28, 49-75) on the engine: the LayerNorm runs in the v4
mixing epilogue (`node_layernorm`, sd_graph_linear_v4.hip), after the Ĝ mixing and before FiLM.

Fixture: tests/golden/layernorm_T10.npz (gen_golden.py gen_layernorm, which ran the reference):
README Denoiser J = 16, release H36M J = 16 and release AMASS J = 21 (two 16-node mixing blocks),
T = 10 with supplied noise.  Tolerance 1e-4 absolute (BASELINE.json north_star)."""
import numpy as np
import pytest
import torch

from conftest import LAYERNORM_MODELS, build_layernorm_diffusion, golden, layernorm_case

pytestmark = pytest.mark.gpu
TOL = 1e-4


def _close(a, ref, tol=TOL):
    a = a.detach().float().cpu().numpy()
    assert a.shape == ref.shape, (a.shape, ref.shape)
    err = float(np.abs(a - ref).max())
    assert err < tol, err


@pytest.mark.parametrize("model", LAYERNORM_MODELS)
def test_layernorm_matches_reference(model, cuda):
    z = golden("layernorm_T10")
    d = build_layernorm_diffusion(model, z, cuda)
    _, _, xc, start, samp, _ = layernorm_case(model, z)
    B = start.shape[0]
    kw = {} if xc is None else {"x_cond": xc.to(cuda)}
    _close(d.engine.denoiser_forward(start.to(cuda), int(z["fwd_t"]), kw.get("x_cond")), z[f"{model}_fwd"])
    for graph in (False, True):
        d.engine.enable_graph(graph)
        img, (_, _, mean_t) = d.sample(batch_size=B, start_noise=start.to(cuda), sampling_noise=samp.to(cuda),
                                       return_sampling_noise=True, **kw)
        _close(img, z[f"{model}_img"])
        _close(mean_t, z[f"{model}_mean_t"])


@pytest.mark.parametrize("model", ["h36m16", "amass21"])
def test_layernorm_routes_bitwise(model, cuda):
    """The LayerNorm lives in the split route's mixing phase: SD_OPT_SPLIT_ROUTE 1 (never split) still
    takes the auto split route for the Block layers, and the small-batch (2) and tiled (3) GEMM
    phases give bitwise equal chains; 3 row chains equal 1; half and bf16 precision sample close to it."""
    z = golden("layernorm_T10")
    d = build_layernorm_diffusion(model, z, cuda)
    J = int(z[f"{model}_corr"].shape[0])
    xc = (torch.rand((8, J, 96), generator=torch.Generator().manual_seed(9)) * 2 - 1).to(cuda)
    ref = None
    for route, chains in ((1, 1), (2, 1), (3, 1), (3, 3), (0, 0)):
        d.engine.set_option("split_route", route)
        d.engine.set_option("row_chains", chains)
        out = d.engine.sample_loop(400, x_cond=xc, seed=4, graph=True)[0].clone()
        torch.cuda.synchronize()
        assert torch.isfinite(out).all()
        if ref is None:
            ref = out
        else:
            assert torch.equal(out, ref), (route, chains, float((out - ref).abs().max()))
    d.engine.set_option("split_route", 0)
    for prec, tol in (("half", 0.05), ("bf16", 0.15)):  # reduced precision: the tiled route, LayerNorm kept
        d.engine.set_precision(prec)
        lo = d.engine.sample_loop(400, x_cond=xc, seed=4, graph=True)[0].float()
        torch.cuda.synchronize()
        assert torch.isfinite(lo).all() and float((lo - ref).abs().max()) < tol, (prec, float((lo - ref).abs().max()))
    d.engine.set_precision("f32")
