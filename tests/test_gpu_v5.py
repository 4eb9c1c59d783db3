"""GPU: the J > 21 mixing pass on the matrix cores (k_gl5_mixm, sd_graph_linear_v5.hip) against the
per-column VALU form (k_gl5_mix) it replaces -- bitwise, over whole sampling chains of the MANO
Denoisers (config 3: J = 51 and the hip-included J = 52), row counts that leave ragged 8-row
workgroups, f32 mode (reference op: graph_structural.py:30-43, G-hat mixing of StaticGraphLinear;
the oracle parity of the chain is test_gpu_parity.py's release_mano51 / release_mano52 goldens)."""
import pytest
import torch

from skeletondiffusion_amd import _lib

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg,batch", [("mano51", 3), ("mano51", 1), ("mano52", 2)])
def test_v5_mix_mfma_bitwise_vs_valu(cfg, batch, cuda):
    from bench import build_config

    d, x_cond, rows = build_config(cfg, cuda, T=10, batch=batch)
    eng = d.engine
    res = {}
    for v in (1, 0):  # SD_OPT_V5_MIX: 1 the VALU form, 0 (default) the matrix cores
        eng.set_option("v5_mix", v)
        a = eng.sample_loop(rows, x_cond=x_cond, seed=5, record=(True, False), graph=False)
        torch.cuda.synchronize()
        res[v] = [t.clone() for t in (a[0], a[3])]  # img, mean_t
    for name, x, y in zip(("img", "mean_t"), res[0], res[1]):
        assert torch.equal(x, y), (name, float((x - y).abs().max()))
    assert eng.get_option("v5_mix") == 0
    with pytest.raises(_lib.SkelDiffError):
        eng.set_option("v5_mix", 2)


@pytest.mark.parametrize("cfg,batch", [("mano51", 3), ("mano52", 2), ("mano51", 64)])
def test_attention_mix_bitwise_vs_separate_pass(cfg, batch, cuda):
    """k_attention_mix at J = 51 / 52 (option 2: the to_qkv layer's G-hat mixing inside the
    attention kernel, the pre-mix Y in the qkv buffer, graph_structural.py:30-43) against the
    separate mixing pass + the padded k_attention (option 3), over whole sampling chains
    (reference op: attention.py:122-136) -- bitwise.  64 sequences = the config-3 batch (3,200
    rows, three row chains, hipGraph) as benched."""
    from bench import build_config

    d, x_cond, rows = build_config(cfg, cuda, T=10 if batch < 64 else 3, batch=batch)
    eng = d.engine
    res = {}
    for v in (2, 3, 0):  # SD_OPT_ATTENTION: 2 mixing in the kernel, 3 separate pass + padded, 0 auto (2)
        eng.set_option("attention", v)
        a = eng.sample_loop(rows, x_cond=x_cond, seed=6, record=(True, False), graph=batch >= 64)
        torch.cuda.synchronize()
        res[v] = [t.clone() for t in (a[0], a[3])]  # img, mean_t
        assert bool(eng.get_option("last_route") & 1024) == (v in (0, 2)), (v, "k_attention_mix")
    assert eng.get_option("last_route") & 128, "the separate k_attention did not run"
    for v in (2, 3):
        for name, x, y in zip(("img", "mean_t"), res[0], res[v]):
            assert torch.equal(x, y), (v, name, float((x - y).abs().max()))
    assert eng.get_option("attention") == 0
    for bad in (1, 4):  # 1: the 48-node tail form ABI 3 removed (measured 1 % slower)
        with pytest.raises(_lib.SkelDiffError):
            eng.set_option("attention", bad)
