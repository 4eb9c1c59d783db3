"""Training-side StaticGraphLinear on HIP (SURVEY.md §8f "next" #4; csrc/sd_train.hip,
skeletondiffusion_amd/training.py).

Kernel parity: forward y and the backward's dx / dW / dbias / dG against float64 torch autograd
over the reference's GraphLinear math (graph_structural.py:30-43: per-type W, bias before the
G-hat mixing, G-hat = G / rowsum|G|), at the Denoiser's shapes (per-type H->H, 2H->H, to_qkv
H->768, README shared weights) and ragged / empty / one-row batches.  Tolerance: max |diff| <=
2e-5 x max |reference| (f32 products, f32 accumulate over <= a few thousand terms).
Training step parity: the release Denoiser's p_losses on the device (HIP graph-linears) against
the reference's own loss (golden fixture) and every parameter's gradient against the CPU torch
path of the same module."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import build_release_diffusion, golden, release_inputs
from skeletondiffusion_amd import synthetic, training
from skeletondiffusion_amd.core.network.layers import StaticGraphLinear

REL_TOL = 2e-5


def _ref_graph_linear(x, W, b, G, types, learn):
    gh = F.normalize(G, p=1.0, dim=1) if learn else G
    if types is not None:
        z = torch.einsum("noi,rni->rno", W[types], x)
        if b is not None:
            z = z + b[types]
    else:
        z = x @ W.t()
        if b is not None:
            z = z + b
    return gh.matmul(z)


def _close(got, ref, what):
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    scale = float(ref.abs().max()) if ref.numel() else 0.0
    err = float((got - ref).abs().max()) if ref.numel() else 0.0
    assert err <= REL_TOL * max(scale, 1e-30) + 1e-12, f"{what}: max |diff| {err:.3e} vs max |ref| {scale:.3e}"


CASES = [  # J, K, N, n_types (0 = shared), bias, learn_influence, rows
    (16, 192, 192, 10, True, True, 257),
    (16, 192, 768, 10, False, True, 64),
    (21, 384, 192, 13, True, True, 100),
    (17, 192, 96, 9, True, True, 65),
    (51, 192, 96, 43, True, True, 33),
    (16, 96, 96, 0, True, False, 8),
    (16, 192, 192, 10, True, True, 1),
]


@pytest.mark.gpu
@pytest.mark.parametrize("J,K,N,nt,bias,learn,rows", CASES)
def test_gl_train_kernel_vs_autograd(J, K, N, nt, bias, learn, rows):
    g = torch.Generator().manual_seed(J * 1000 + K + N + rows)
    x = torch.rand(rows, J, K, generator=g, dtype=torch.float64) * 2 - 1
    W = (torch.rand((nt, N, K) if nt else (N, K), generator=g, dtype=torch.float64) * 2 - 1) / K ** 0.5
    b = (torch.rand((nt, N) if nt else (N,), generator=g, dtype=torch.float64) - 0.5) if bias else None
    G = torch.eye(J, dtype=torch.float64) + 0.1 * torch.rand(J, J, generator=g, dtype=torch.float64)
    types = torch.randint(0, nt, (J,), generator=g) if nt else None
    if nt:
        types[:nt] = torch.arange(nt)[: min(nt, J)]
    dy = torch.rand(rows, J, N, generator=g, dtype=torch.float64) * 2 - 1

    leaves = [t.clone().requires_grad_(True) for t in (x, W, G)] + ([b.clone().requires_grad_(True)] if bias else [])
    y_ref = _ref_graph_linear(leaves[0], leaves[1], leaves[3] if bias else None, leaves[2], types, learn)
    y_ref.backward(dy)

    dev = torch.device("cuda:0")
    dl = [t.float().to(dev).requires_grad_(True) for t in (x, W, G)] + \
         ([b.float().to(dev).requires_grad_(True)] if bias else [])
    gh = F.normalize(dl[2], p=1.0, dim=1) if learn else dl[2]
    y = training.graph_linear(dl[0], dl[1], dl[3] if bias else None, gh,
                              None if types is None else types.to(dev))
    y.backward(dy.float().to(dev))
    torch.cuda.synchronize()
    _close(y, y_ref, "y")
    _close(dl[0].grad, leaves[0].grad, "dx")
    _close(dl[1].grad, leaves[1].grad, "dW")
    if learn:
        _close(dl[2].grad, leaves[2].grad, "dG")
    if bias:
        _close(dl[3].grad, leaves[3].grad, "dbias")


@pytest.mark.gpu
def test_gl_train_empty_batch():
    dev = torch.device("cuda:0")
    x = torch.zeros(0, 16, 64, device=dev, requires_grad=True)
    W = torch.rand(3, 32, 64, device=dev, requires_grad=True)
    b = torch.rand(3, 32, device=dev, requires_grad=True)
    G = torch.eye(16, device=dev, requires_grad=True)
    types = (torch.arange(16) % 3).to(dev)
    y = training.graph_linear(x, W, b, G, types)
    assert y.shape == (0, 16, 32)
    y.sum().backward()
    torch.cuda.synchronize()
    assert x.grad.shape == x.shape
    assert float(W.grad.abs().max()) == 0.0 and float(b.grad.abs().max()) == 0.0 and float(G.grad.abs().max()) == 0.0


@pytest.mark.gpu
def test_gl_train_deterministic():
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(7)
    x = torch.rand(300, 16, 192, generator=g).to(dev).requires_grad_(True)
    W = torch.rand(10, 192, 192, generator=g).to(dev).requires_grad_(True)
    G = torch.rand(16, 16, generator=g).to(dev).requires_grad_(True)
    types = (torch.arange(16) % 10).to(dev)
    grads = []
    for _ in range(2):
        for t in (x, W, G):
            t.grad = None
        training.graph_linear(x, W, None, G, types).pow(2).sum().backward()
        grads.append([t.grad.clone() for t in (x, W, G)])
    for a, c in zip(*grads):
        assert torch.equal(a, c)


def _grad_fn_names(t):
    seen, out, stack = set(), set(), [t.grad_fn]
    while stack:
        f = stack.pop()
        if f is None or f in seen:
            continue
        seen.add(f)
        out.add(type(f).__name__)
        stack.extend(n for n, _ in f.next_functions)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["release_h36m16_T10", "release_amass21_T10"])
def test_release_training_step_on_hip(name):
    z = golden(name)
    xcs, fu, start, _ = release_inputs(z)
    xc = xcs.repeat_interleave(fu, 0)
    B, J = start.shape[0], start.shape[1]
    T = int(z["T"])
    t_train = torch.arange(B) % T
    noise = torch.from_numpy(synthetic.normal((B, J, 96), 24))
    xs = torch.from_numpy(synthetic.uniform((B, J, 96), 25))

    d_cpu = build_release_diffusion(z)
    loss_c, _, _ = d_cpu.p_losses(xs, t_train, noise=noise, x_cond=xc)
    loss_c.mean().backward()

    dev = torch.device("cuda:0")
    d_gpu = build_release_diffusion(z, device=dev)
    assert training.hip_training_enabled()
    loss_g, lw, mout = d_gpu.p_losses(xs.to(dev), t_train.to(dev), noise=noise.to(dev), x_cond=xc.to(dev))
    assert "GraphLinearFunctionBackward" in _grad_fn_names(loss_g), "HIP graph-linear not on the training path"
    assert "AttentionCoreFunctionBackward" in _grad_fn_names(loss_g), "HIP attention core not on the training path"
    assert "FilmTanhFunctionBackward" in _grad_fn_names(loss_g), "HIP FiLM + tanh not on the training path"
    assert "RMSNormFunctionBackward" in _grad_fn_names(loss_g), "HIP RMSNorm not on the training path"
    assert "MahalanobisLossFunctionBackward" in _grad_fn_names(loss_g), "HIP loss not on the training path"
    if d_gpu.model.init_lin.learn_influence:
        assert "L1NormRowsFunctionBackward" in _grad_fn_names(loss_g), "HIP G-hat not on the training path"
    loss_g.mean().backward()
    torch.cuda.synchronize()
    # the reference's own loss (gen_golden.py, reference p_losses on CPU)
    np.testing.assert_allclose(loss_g.detach().cpu().numpy(), z["train_loss"], atol=1e-5, rtol=1e-5)
    np.testing.assert_allclose(mout.detach().cpu().numpy(), z["train_model_out"], atol=1e-5, rtol=0)
    pc = dict(d_cpu.named_parameters())
    n_checked = 0
    for k, p in d_gpu.named_parameters():
        if pc[k].grad is None:
            assert p.grad is None or float(p.grad.abs().max()) == 0.0, k
            continue
        # gradients of a mean L1 loss: compare against the CPU path's scale per tensor
        got, ref = p.grad.double().cpu(), pc[k].grad.double()
        err, scale = float((got - ref).abs().max()), float(ref.abs().max())
        assert err <= 1e-3 * scale + 1e-9, f"{k}: max |diff| {err:.3e} vs max |ref| {scale:.3e}"
        n_checked += 1
    assert n_checked > 100


def test_graph_linear_needs_device_tensors():
    x = torch.zeros(2, 16, 8)
    with pytest.raises(ValueError):
        training.graph_linear(x, torch.zeros(4, 8), None, torch.eye(16), None)


def test_cpu_module_keeps_torch_path():
    m = StaticGraphLinear(8, 4, num_nodes=5, node_types=torch.tensor([0, 1, 0, 2, 1]), learn_influence=True)
    x = torch.rand(3, 5, 8)
    y = m(x)
    ref = _ref_graph_linear(x, m.weight, m.bias, m.G, m.node_type_index, True)
    torch.testing.assert_close(y, ref)
    prev = training.set_hip_training(False)
    assert prev is True and not training.hip_training_enabled()
    training.set_hip_training(prev)


def test_gl_train_abi_validation_on_host():
    """Argument checks of the training ABI run before any device work (no GPU needed)."""
    from skeletondiffusion_amd import _lib
    L = _lib.lib()
    ws = L.sd_gl_train_workspace_bytes(1024, 16, 192, 192, 10)
    # dz (rows, J, N) plus the largest partial buffer (dW split partials)
    assert ws >= 1024 * 16 * 192 * 4 + 192 * 192 * 10 * 4
    assert L.sd_gl_train_workspace_bytes(2048, 16, 192, 192, 10) > ws
    assert L.sd_gl_train_workspace_bytes(-1, 16, 192, 192, 10) == 0
    assert L.sd_gl_train_forward(None, None, None, None, 0, None, 4, 0, 8, 8, None, None, None) < 0   # J = 0
    assert b"J" in L.sd_last_error()
    assert L.sd_gl_train_forward(None, None, None, None, 0, None, 4, 65, 8, 8, None, None, None) < 0  # J > 64
    assert L.sd_gl_train_forward(None, None, None, None, 0, None, 0, 16, 8, 8, None, None, None) == 0  # empty
    assert L.sd_gl_train_forward(None, None, None, None, 0, None, 4, 16, 8, 8, None, None, None) < 0   # null buffers
    assert L.sd_gl_train_backward(None, None, None, None, None, 0, None, 4, 16, 8, 8, None, None, None, None,
                                  None, 0, None) < 0                                                  # null input


def _ref_attention(qkv, heads, dh, scale):
    """The reference's attention core (attention.py:122-136) on (rows, J, 3 heads dh)."""
    b, n, _ = qkv.shape
    q, k, v = (c.reshape(b, n, heads, dh).permute(0, 2, 3, 1) for c in qkv.chunk(3, dim=-1))
    attn = torch.einsum("bhcn,bhcj->bhnj", q * scale, k).softmax(dim=-1)
    out = torch.einsum("bhnj,bhdj->bhnd", attn, v)
    return out.permute(0, 2, 1, 3).reshape(b, n, heads * dh)


@pytest.mark.gpu
@pytest.mark.parametrize("J,heads,dh,rows", [(16, 8, 32, 300), (17, 8, 32, 33), (21, 8, 32, 7), (51, 8, 32, 5),
                                              (52, 2, 64, 3), (64, 4, 64, 2), (16, 8, 32, 1), (16, 8, 32, 0)])
def test_attention_core_vs_autograd(J, heads, dh, rows):
    """sd_attn_train_forward / _backward (training.AttentionCoreFunction) against float64 autograd
    of the reference formula: out, and dqkv from a random upstream gradient."""
    g = torch.Generator().manual_seed(J * 100 + heads + rows)
    qkv = torch.randn(rows, J, 3 * heads * dh, generator=g, dtype=torch.float64)
    dout = torch.randn(rows, J, heads * dh, generator=g, dtype=torch.float64)
    scale = dh ** -0.5
    ref_in = qkv.clone().requires_grad_(True)
    ref = _ref_attention(ref_in, heads, dh, scale)
    (ref * dout).sum().backward()
    dev = torch.device("cuda:0")
    x = qkv.float().to(dev).requires_grad_(True)
    out = training.attention_core(x, heads, dh, scale)
    out.backward(dout.float().to(dev))
    torch.cuda.synchronize()
    assert out.shape == (rows, J, heads * dh)
    _close(out, ref, "out")
    _close(x.grad, ref_in.grad, "dqkv")


def test_attention_core_abi_validation_on_host():
    """Argument checks of the attention training ABI run before any device work."""
    from skeletondiffusion_amd import _lib
    L = _lib.lib()
    assert L.sd_attn_train_forward(None, None, 4, 0, 8, 32, 1.0, None) < 0       # J = 0
    assert b"J" in L.sd_last_error()
    assert L.sd_attn_train_forward(None, None, 4, 65, 8, 32, 1.0, None) < 0      # J > 64
    assert L.sd_attn_train_forward(None, None, 4, 16, 8, 65, 1.0, None) < 0      # dim_head > 64
    assert L.sd_attn_train_forward(None, None, 4, 16, 8, 32, 1.0, None) < 0      # null buffers
    assert L.sd_attn_train_backward(None, None, None, 4, 16, 8, 32, 1.0, None) < 0
    with pytest.raises(ValueError):
        training.attention_core(torch.zeros(2, 16, 96), 1, 32, 1.0)                # host tensor


@pytest.mark.gpu
@pytest.mark.parametrize("rows,J,C", [(257, 16, 192), (5, 21, 192), (1, 51, 96), (0, 16, 192)])
def test_film_tanh_vs_autograd(rows, J, C):
    """sd_film_tanh_forward / _backward (training.FilmTanhFunction) against float64 autograd of the
    reference's Block epilogue x * (scale + 1) + shift -> tanh (attention.py:67-75)."""
    g = torch.Generator().manual_seed(rows + J + C)
    y = torch.randn(rows, J, C, generator=g, dtype=torch.float64)
    ss = torch.randn(rows, 1, 2 * C, generator=g, dtype=torch.float64) * 0.5
    dout = torch.randn(rows, J, C, generator=g, dtype=torch.float64)
    yr, sr = y.clone().requires_grad_(True), ss.clone().requires_grad_(True)
    sc, sh = sr.chunk(2, dim=-1)
    ref = torch.tanh(yr * (sc + 1) + sh)
    (ref * dout).sum().backward()
    dev = torch.device("cuda:0")
    yg, sg = y.float().to(dev).requires_grad_(True), ss.float().to(dev).requires_grad_(True)
    out = training.film_tanh(yg, sg)
    out.backward(dout.float().to(dev))
    torch.cuda.synchronize()
    _close(out, ref, "out")
    _close(yg.grad, yr.grad, "dy")
    _close(sg.grad, sr.grad, "dss")


@pytest.mark.gpu
@pytest.mark.parametrize("J,zero_row", [(16, False), (21, True), (51, False), (64, True), (1, False)])
def test_l1norm_rows_vs_autograd(J, zero_row):
    """sd_l1norm_rows_forward / _backward (training.L1NormRowsFunction) against float64 autograd of
    F.normalize(G, p=1, dim=1) (graph_structural.py:107), a zero row included (the eps clamp)."""
    g = torch.Generator().manual_seed(J)
    G = torch.randn(J, J, generator=g, dtype=torch.float64)
    if zero_row:
        G[J // 2] = 0.0
    dout = torch.randn(J, J, generator=g, dtype=torch.float64)
    Gr = G.clone().requires_grad_(True)
    ref = F.normalize(Gr, p=1.0, dim=1)
    (ref * dout).sum().backward()
    dev = torch.device("cuda:0")
    Gg = G.float().to(dev).requires_grad_(True)
    out = training.l1norm_rows(Gg)
    out.backward(dout.float().to(dev))
    torch.cuda.synchronize()
    _close(out, ref, "ghat")
    _close(Gg.grad, Gr.grad, "dG")


@pytest.mark.gpu
def test_l1norm_rows_batched_vs_autograd():
    """Several G in one launch each way (training.l1norm_rows_many, what Denoiser.forward uses):
    each output and gradient equals float64 autograd of its own F.normalize; an output with no
    upstream gradient contributes zeros."""
    J, L = 21, 5
    g = torch.Generator().manual_seed(99)
    Gs = [torch.randn(J, J, generator=g, dtype=torch.float64) for _ in range(L)]
    Gs[2][3] = 0.0
    douts = [torch.randn(J, J, generator=g, dtype=torch.float64) for _ in range(L)]
    dev = torch.device("cuda:0")
    Gg = [G.float().to(dev).requires_grad_(True) for G in Gs]
    outs = training.l1norm_rows_many(Gg)
    sum((o * d.float().to(dev)).sum() for k, (o, d) in enumerate(zip(outs, douts)) if k != 4).backward()
    torch.cuda.synchronize()
    for k in range(L):
        Gr = Gs[k].clone().requires_grad_(True)
        ref = F.normalize(Gr, p=1.0, dim=1)
        (ref * (douts[k] if k != 4 else torch.zeros_like(douts[k]))).sum().backward()
        _close(outs[k], ref, f"ghat[{k}]")
        _close(Gg[k].grad, Gr.grad, f"dG[{k}]")


@pytest.mark.gpu
@pytest.mark.parametrize("rows,J,C", [(257, 16, 192), (5, 21, 192), (1, 51, 96), (3, 16, 1024), (0, 16, 192)])
def test_rmsnorm_vs_autograd(rows, J, C):
    """sd_rmsnorm_forward / _backward (training.RMSNormFunction) against float64 autograd of the
    reference's RMSNorm (attention.py:30-36), one all-zero vector included (the eps clamp)."""
    g = torch.Generator().manual_seed(rows * 7 + J + C)
    x = torch.randn(rows, J, C, generator=g, dtype=torch.float64)
    if rows:
        x[0, J - 1] = 0.0
    gain = 1 + 0.3 * torch.randn(1, 1, C, generator=g, dtype=torch.float64)
    dout = torch.randn(rows, J, C, generator=g, dtype=torch.float64)
    xr, gr = x.clone().requires_grad_(True), gain.clone().requires_grad_(True)
    ref = F.normalize(xr, dim=-1) * gr * (C ** 0.5)
    (ref * dout).sum().backward()
    dev = torch.device("cuda:0")
    xg, gg = x.float().to(dev).requires_grad_(True), gain.float().to(dev).requires_grad_(True)
    out = training.rmsnorm(xg, gg, C ** 0.5)
    out.backward(dout.float().to(dev))
    torch.cuda.synchronize()
    assert out.shape == (rows, J, C) and gg.grad.shape == (1, 1, C)
    _close(out, ref, "out")
    _close(xg.grad, xr.grad, "dx")
    if rows:
        _close(gg.grad, gr.grad, "dg")
    else:
        assert float(gg.grad.abs().max()) == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("rows,J,F_,pred_noise,mse", [(257, 16, 96, True, False), (33, 21, 96, False, False),
                                                      (5, 51, 96, True, True), (2, 64, 256, False, True),
                                                      (1, 17, 96, True, False), (0, 16, 96, True, False)])
def test_mahalanobis_loss_vs_autograd(rows, J, F_, pred_noise, mse):
    """sd_mahalanobis_loss_forward / _backward (training.MahalanobisLossFunction) against float64
    autograd of the reference's loss_funct + per-row mean (nonisotropic.py:177-190,
    base.py:297-298): the loss and d model_out / d target from a random per-row upstream gradient."""
    g = torch.Generator().manual_seed(rows + 13 * J + F_ + 2 * int(mse))
    T = 10
    mo = torch.randn(rows, J, F_, generator=g, dtype=torch.float64)
    tg = torch.randn(rows, J, F_, generator=g, dtype=torch.float64)
    S = torch.randn(T, J, J, generator=g, dtype=torch.float64) / J ** 0.5
    t = torch.randint(0, T, (rows,), generator=g)
    dl = torch.rand(rows, generator=g, dtype=torch.float64) + 0.5
    mr, tr = mo.clone().requires_grad_(True), tg.clone().requires_grad_(True)
    diff = tr - mr if pred_noise else mr - tr
    m = (S[t] @ diff).abs()
    ref = (m ** 2 if mse else m).reshape(rows, J * F_).mean(dim=1)
    (ref * dl).sum().backward()
    dev = torch.device("cuda:0")
    mg, tgg = mo.float().to(dev).requires_grad_(True), tg.float().to(dev).requires_grad_(True)
    loss = training.mahalanobis_loss(mg, tgg, S.float().to(dev), t.to(dev), pred_noise, mse)
    loss.backward(dl.float().to(dev))
    torch.cuda.synchronize()
    assert loss.shape == (rows,)
    _close(loss, ref, "loss")
    _close(mg.grad, mr.grad, "d model_out")
    _close(tgg.grad, tr.grad, "d target")


def test_new_training_abi_validation_on_host():
    """Argument checks of the G-hat / RMSNorm / loss training ABI run before any device work."""
    from skeletondiffusion_amd import _lib
    L = _lib.lib()
    assert L.sd_l1norm_rows_forward(None, None, 0, 1, 1e-12, None) < 0       # J = 0
    assert b"J" in L.sd_last_error()
    assert L.sd_l1norm_rows_forward(None, None, 65, 1, 1e-12, None) < 0      # J > 64
    assert L.sd_l1norm_rows_forward(None, None, 16, -1, 1e-12, None) < 0     # count < 0
    assert L.sd_l1norm_rows_forward(None, None, 16, 0, 1e-12, None) == 0     # nothing to do
    assert L.sd_l1norm_rows_forward(None, None, 16, 1, 1e-12, None) < 0      # null buffers
    assert L.sd_l1norm_rows_backward(None, None, None, 16, 1, 1e-12, None) < 0
    assert L.sd_rmsnorm_workspace_bytes(1024 * 16, 192) == 1024 * 192 * 4    # one dg partial per 16 vectors
    assert L.sd_rmsnorm_workspace_bytes(-1, 192) == 0
    assert L.sd_rmsnorm_forward(None, None, None, None, 4, 1025, 1.0, 1e-12, None) < 0   # C > 1024
    assert L.sd_rmsnorm_forward(None, None, None, None, 0, 192, 1.0, 1e-12, None) == 0   # empty
    assert L.sd_rmsnorm_forward(None, None, None, None, 4, 192, 1.0, 1e-12, None) < 0    # null buffers
    assert L.sd_rmsnorm_backward(None, None, None, None, None, None, 4, 192, 1.0, 1e-12, None, 0, None) < 0
    assert L.sd_mahalanobis_loss_forward(None, None, None, None, 10, 4, 65, 96, 1, 0, None, None) < 0   # J > 64
    assert L.sd_mahalanobis_loss_forward(None, None, None, None, 10, 4, 16, 257, 1, 0, None, None) < 0  # F > 256
    assert L.sd_mahalanobis_loss_forward(None, None, None, None, 0, 4, 16, 96, 1, 0, None, None) < 0    # T < 1
    assert L.sd_mahalanobis_loss_forward(None, None, None, None, 10, 0, 16, 96, 1, 0, None, None) == 0  # empty
    assert L.sd_mahalanobis_loss_backward(None, None, None, None, 10, None, 4, 16, 96, 1, 0, None, None) < 0
    with pytest.raises(ValueError):
        training.rmsnorm(torch.zeros(2, 16, 8), torch.ones(8), 8 ** 0.5)      # host tensor
    with pytest.raises(ValueError):
        training.l1norm_rows(torch.eye(4))
    with pytest.raises(ValueError):
        training.mahalanobis_loss(torch.zeros(2, 16, 96), torch.zeros(2, 16, 96), torch.zeros(3, 16, 16),
                                  torch.zeros(2, dtype=torch.long), True, False)


@pytest.mark.gpu
def test_mahalanobis_loss_out_of_range_timestep_is_nan():
    """A timestep outside [0, T) reads no table row (advisor finding, round 3): that row's loss and
    gradient are NaN, the other rows are unaffected."""
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(5)
    T, J, F_ = 4, 16, 96
    S = (torch.randn(T, J, J, generator=g) / J ** 0.5).to(dev)
    mo = torch.randn(3, J, F_, generator=g).to(dev).requires_grad_(True)
    tg = torch.randn(3, J, F_, generator=g).to(dev)
    t = torch.tensor([1, T, -1], device=dev)
    loss = training.mahalanobis_loss(mo, tg, S, t, True, False)
    loss.sum().backward()
    torch.cuda.synchronize()
    assert torch.isfinite(loss[0]) and torch.isnan(loss[1]) and torch.isnan(loss[2])
    assert torch.isfinite(mo.grad[0]).all() and torch.isnan(mo.grad[1]).all() and torch.isnan(mo.grad[2]).all()
