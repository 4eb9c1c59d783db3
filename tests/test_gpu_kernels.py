"""Per-kernel numerics on the GPU: each HIP kernel (through the ABI test hooks) against a plain
PyTorch fp32 CPU computation of the same op, on random inputs, across the J / N / K shapes the
configs use (and odd ones that take the generic paths)."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from skeletondiffusion_amd import _lib

pytestmark = pytest.mark.gpu


def _gl_reference(x1, x2, W, bias, types, ghat, film, act, res, rms, div):
    B = x1.shape[0] * div
    x1r = x1.repeat_interleave(div, 0)
    x = torch.cat([x1r, x2], -1) if x2 is not None else x1r
    w = W[types]                                              # (J, N, K)
    y = torch.einsum("jnk,bjk->bjn", w.double(), x.double())
    if rms:
        y = y / x1r.double().norm(dim=-1, keepdim=True).clamp_min(1e-12)
    if bias is not None:
        y = y + bias[types].double()
    z = ghat.double() @ y
    if film is not None:
        N = W.shape[1]
        z = z * (film[:N].double() + 1) + film[N:].double()
    if act:
        z = torch.tanh(z)
    if res is not None:
        z = z + res.double()
    assert z.shape[0] == B
    return z.float()


def to_blocked(t):
    """(B, J, F) -> the v4 row-blocked layout, flat: per 32-row block and node, [F/8][2][32][4]."""
    B, J, F = t.shape
    Bp = (B + 31) // 32 * 32
    tp = torch.zeros(Bp, J, F, dtype=t.dtype)
    tp[:B] = t
    return tp.view(Bp // 32, 32, J, F // 8, 2, 4).permute(0, 2, 3, 4, 1, 5).contiguous().view(-1)


def from_blocked(flat, B, J, F):
    Bp = (B + 31) // 32 * 32
    return flat.view(Bp // 32, J, F // 8, 2, 32, 4).permute(0, 4, 1, 2, 3, 5).reshape(Bp, J, F)[:B]


def test_blocked_layout_helpers():
    t = torch.arange(67 * 3 * 16, dtype=torch.float32).view(67, 3, 16)
    b = to_blocked(t)
    assert b.numel() == 96 * 3 * 16
    assert torch.equal(from_blocked(b, 67, 3, 16), t)
    # element (row 33, node 2, feature 13): block 1, octet 1, half 1, row 1, lane 1
    off = ((1 * 3 + 2) * 16 * 32) + 1 * 256 + 1 * 128 + 1 * 4 + 1
    assert b[off] == t[33, 2, 13]


def _run_gl(dev, x1, x2, W, bias, types, ghat, film, act, res, rms, div):
    B = x1.shape[0] * div
    J, N = x1.shape[1], W.shape[1]
    t = lambda a: None if a is None else a.to(dev).contiguous()  # noqa: E731
    g = {k: t(v) for k, v in dict(x1=x1, x2=x2, W=W, bias=bias, ghat=ghat, film=film, res=res).items()}
    out = torch.full((B, J, N), float("nan"), device=dev)
    nt = (ctypes.c_int64 * J)(*types.tolist())
    p = lambda a: None if a is None else a.data_ptr()  # noqa: E731
    _lib.check(_lib.lib().sd_test_graph_linear(p(g["x1"]), x1.shape[2], div, p(g["x2"]),
                                               0 if x2 is None else x2.shape[2], p(g["W"]), p(g["bias"]), nt,
                                               p(g["ghat"]), p(g["film"]), act, p(g["res"]), out.data_ptr(), B, J,
                                               N, int(rms), 0))
    torch.cuda.synchronize()
    return out.cpu()


CASES = [  # (J, n_types, K1, K2, N, div, bias, film, act, res, rms)
    (16, 1, 96, 0, 96, 1, True, False, 0, False, False),      # README shared weights
    (16, 10, 96, 96, 192, 4, True, False, 0, False, False),    # init_lin with x_cond broadcast
    (16, 10, 192, 0, 192, 1, True, True, 1, False, False),    # ResnetBlock block1 (FiLM + tanh)
    (16, 10, 192, 0, 192, 1, True, False, 1, True, False),    # block2 (tanh + residual)
    (16, 10, 192, 0, 768, 1, False, False, 0, False, True),   # to_qkv with RMSNorm scale
    (16, 10, 256, 0, 192, 1, False, False, 0, True, False),   # to_out + residual
    (16, 10, 192, 192, 192, 1, False, False, 0, False, False),  # final res_linear on cat(x, r)
    (16, 10, 192, 0, 96, 1, True, False, 0, False, False),    # final_glin
    (17, 9, 192, 0, 192, 1, True, True, 1, False, False),
    (21, 13, 96, 96, 192, 50, True, False, 0, False, False),
    (21, 13, 192, 0, 768, 1, False, False, 0, False, True),
    (51, 43, 192, 0, 192, 1, True, True, 1, True, False),
    (51, 43, 192, 0, 768, 1, False, False, 0, False, True),
    (5, 3, 96, 0, 96, 1, True, False, 0, False, False),       # generic JM=8 path
    (12, 4, 192, 0, 192, 1, True, True, 1, True, True),       # generic JM=16 path, everything on
    (33, 7, 96, 0, 192, 1, True, False, 1, False, False),     # generic JM=64 path
    # J > 21 (v5's split GEMM phase) with an odd chunk count: latent_dim 16 / 48, cond_dim 0
    (33, 7, 16, 0, 96, 1, True, False, 0, False, False),
    (33, 7, 48, 0, 96, 1, True, False, 0, False, False),
    (51, 43, 48, 0, 192, 1, True, False, 1, True, False),
]


@pytest.mark.parametrize("J,nty,K1,K2,N,div,has_bias,has_film,act,has_res,rms", CASES)
@pytest.mark.parametrize("Bseq", [64, 67])
def test_graph_linear_kernel(J, nty, K1, K2, N, div, has_bias, has_film, act, has_res, rms, Bseq, cuda):
    _check_gl(J, nty, K1, K2, N, div, has_bias, has_film, act, has_res, rms, Bseq, cuda)


@pytest.fixture
def kernel_variant():
    """Select a graph-linear generation / v4 tile for one test, restoring auto afterwards."""
    L = _lib.lib()

    def set_(v, tile=0):
        assert L.sd_test_set_kernel_variant(v, tile) >= 0

    yield set_
    L.sd_test_set_kernel_variant(0, 0)


# every v4 tile instantiation for J=16 and the exact-f32 generations on the release shapes
V4_TILES = [0, 412, 421, 821, 811, 812, 813, 822]


@pytest.mark.parametrize("case", [c for c in CASES if c[0] == 16])
@pytest.mark.parametrize("variant,tile", [(4, t) for t in V4_TILES] + [(3, 0), (2, 0), (1, 0)])
def test_graph_linear_generations(case, variant, tile, kernel_variant, cuda):
    kernel_variant(variant, tile)
    _check_gl(*case, 67, cuda)


@pytest.mark.parametrize("case", CASES)
def test_graph_linear_v5(case, kernel_variant, cuda):
    """v5 (node-batched GEMM + mixing pass; the default for J > 21) forced on every shape."""
    kernel_variant(5, 0)
    _check_gl(*case, 67, cuda)


@pytest.fixture
def split_route():
    """Select the split route of the sd_test_graph_linear* hooks for one test, restoring auto."""
    L = _lib.lib()

    def set_(route):
        assert L.sd_test_set_split_route(route) >= 0

    yield set_
    L.sd_test_set_split_route(0)


@pytest.mark.parametrize("route", [2, 3])
def test_split_route_hook_matches_reference(route, split_route, cuda):
    """sd_test_set_split_route: the J <= 21 split routes (k_gl4y / k_gl4t GEMM phase + k_gl4 MODE 2)
    through the kernel test hook, against the float64 reference."""
    split_route(route)
    for case in [c for c in CASES if c[0] in (16, 17, 21) and c[4] % 32 == 0]:
        _check_gl(*case, 67, cuda)


@pytest.mark.parametrize("J,nty,K1,K2,N,has_res,rms", [(16, 10, 192, 0, 192, True, False), (16, 10, 96, 96, 192, False, False),
                                                       (16, 10, 192, 0, 768, False, True), (17, 9, 192, 0, 192, False, False),
                                                       (51, 43, 192, 0, 192, True, False), (51, 43, 192, 0, 768, False, True)])
@pytest.mark.parametrize("route", [2, 3])
def test_graph_linear_out_of_f16_range(J, nty, K1, K2, N, has_res, rms, route, split_route, cuda):
    """Operands the split-f16 products cannot represent (|x| >= 65504: rows scaled by 1e5 and
    1e12): the waves holding them recompute their tiles on exact-f32 MFMA (exact_tile_f32), so
    every row stays within 2e-5 of the float64 reference relative to that row's magnitude; the
    in-range rows of the same launch keep the absolute 2e-5.  J <= 21: the split routes' GEMM
    phases k_gl4y (route 2) and k_gl4t (route 3) + the MODE 2 mixing phase; J = 51: v5, whose GEMM
    phase is k_gl4t / k_gl4y row-major (the route setting does not apply).  The one-kernel tiles
    only flag SD_STATUS_F16_RANGE."""
    if J > 21 and route == 3:
        pytest.skip("v5 picks its GEMM phase itself")
    split_route(route)
    B = 67
    g = torch.Generator().manual_seed(J + N + K1 + K2)
    r = lambda *s: torch.rand(*s, generator=g) * 2 - 1  # noqa: E731
    x1 = r(B, J, K1)
    x1[5] *= 1e5
    x1[40, 3] *= 1e12
    x2 = r(B, J, K2) if K2 else None
    if x2 is not None:
        x2[33, :, 7] = 7e4
    W = r(nty, N, K1 + K2) / (K1 + K2) ** 0.5
    types = torch.arange(J) % nty
    bias = r(nty, N) * 0.1
    ghat = F.normalize(torch.eye(J) + torch.rand(J, J, generator=g) * 0.1, p=1.0, dim=1)
    res = r(B, J, N) if has_res else None
    got = _run_gl(cuda, x1, x2, W, bias, types, ghat, None, 0, res, rms, 1)
    ref = _gl_reference(x1, x2, W, bias, types, ghat, None, 0, res, rms, 1)
    assert torch.isfinite(got).all()
    scale = ref.abs().amax(dim=(1, 2)).clamp_min(1.0)  # per row
    err = ((got - ref).abs().amax(dim=(1, 2)) / scale).max().item()
    assert err < 2e-5, err


def test_kernel_variant_rejects_bad_value():
    L = _lib.lib()
    assert L.sd_test_set_kernel_variant(9, -1) < 0
    assert L.sd_test_set_kernel_variant(0, -1) == 0


def _check_gl(J, nty, K1, K2, N, div, has_bias, has_film, act, has_res, rms, Bseq, cuda):
    g = torch.Generator().manual_seed(J * 1000 + N + K1 + K2 + Bseq)
    B = Bseq if div == 1 else max(1, Bseq // div) * div
    r = lambda *s: torch.rand(*s, generator=g) * 2 - 1  # noqa: E731
    x1 = r(B // div, J, K1)
    x2 = r(B, J, K2) if K2 else None
    W = r(nty, N, K1 + K2) / (K1 + K2) ** 0.5
    types = torch.randint(0, nty, (J,), generator=g)
    types[:nty] = torch.randperm(nty, generator=g)[: min(nty, J)] if nty <= J else types[:nty]
    bias = r(nty, N) * 0.1 if has_bias else None
    G = torch.eye(J) + torch.rand(J, J, generator=g) * 0.1
    ghat = F.normalize(G, p=1.0, dim=1)
    film = r(2 * N) * 0.5 if has_film else None
    res = r(B, J, N) if has_res else None
    got = _run_gl(cuda, x1, x2, W, bias, types, ghat, film, act, res, rms, div)
    ref = _gl_reference(x1, x2, W, bias, types, ghat, film, act, res, rms, div)
    assert torch.isfinite(got).all()
    assert (got - ref).abs().max().item() < 2e-5


@pytest.mark.parametrize("J", [16, 17, 21, 51, 7, 33])
@pytest.mark.parametrize("heads,dh", [(8, 32), (4, 32), (2, 64)])
def test_attention_kernel(J, heads, dh, cuda):
    g = torch.Generator().manual_seed(J + heads)
    B = 37
    hid = heads * dh
    qkv = torch.randn(B, J, 3 * hid, generator=g)
    q, k, v = (c.reshape(B, J, heads, dh).permute(0, 2, 3, 1) for c in qkv.chunk(3, dim=-1))
    sim = torch.einsum("bhcn,bhcj->bhnj", q.double() * dh ** -0.5, k.double())
    ref = torch.einsum("bhnj,bhdj->bhnd", sim.softmax(-1), v.double()).permute(0, 2, 1, 3).reshape(B, J, hid)
    out = torch.full((B, J, hid), float("nan"), device=cuda)
    qd = qkv.to(cuda)
    _lib.check(_lib.lib().sd_test_attention(qd.data_ptr(), out.data_ptr(), B, J, heads, dh, 0))
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()
    assert (out.cpu().double() - ref).abs().max().item() < 2e-5


@pytest.mark.parametrize("J,nty,heads,rms", [(16, 10, 8, True), (16, 1, 4, True), (16, 10, 8, False), (16, 3, 2, True),
                                          (17, 9, 8, True), (21, 13, 8, True), (21, 13, 2, False)])
@pytest.mark.parametrize("B", [64, 67, 704])
@pytest.mark.parametrize("blocked", [False, True])
def test_qkv_attention_fused(J, nty, heads, rms, B, blocked, cuda):
    """Fused to_qkv + attention kernel vs a float64 torch restatement of the two ops (B <= 640:
    the split route's k_gl4y + k_gl4 MODE 3; B = 704: the one-kernel k_gl4 MODE 1)."""
    g = torch.Generator().manual_seed(J * 100 + heads + B + rms)
    K, hid = 192, heads * 32
    r = lambda *s: torch.rand(*s, generator=g) * 2 - 1  # noqa: E731
    x = r(B, J, K)
    W = r(nty, 3 * hid, K) / K ** 0.5
    types = torch.randint(0, nty, (J,), generator=g)
    ghat = F.normalize(torch.eye(J) + torch.rand(J, J, generator=g) * 0.1, p=1.0, dim=1)
    qkv = _gl_reference(x, None, W, None, types, ghat, None, 0, None, rms, 1).double()
    q, k, v = (c.reshape(B, J, heads, 32).permute(0, 2, 3, 1) for c in qkv.chunk(3, dim=-1))
    sim = torch.einsum("bhcn,bhcj->bhnj", q * 32 ** -0.5, k)
    ref = torch.einsum("bhnj,bhdj->bhnd", sim.softmax(-1), v).permute(0, 2, 1, 3).reshape(B, J, hid)
    out = torch.full((B, J, hid), float("nan"), device=cuda)
    nt = (ctypes.c_int64 * J)(*types.tolist())
    xd, Wd, gd = x.to(cuda), W.to(cuda), ghat.to(cuda)
    if blocked:
        xd = to_blocked(x).to(cuda)
        outb = torch.full((to_blocked(torch.zeros(B, J, hid)).numel(),), float("nan"), device=cuda)
    _lib.check(_lib.lib().sd_test_qkv_attention(xd.data_ptr(), K, Wd.data_ptr(), nt, gd.data_ptr(),
                                                (outb if blocked else out).data_ptr(), B, J, heads, int(rms),
                                                9 if blocked else 0, 0))
    torch.cuda.synchronize()
    got = (from_blocked(outb.cpu(), B, J, hid) if blocked else out.cpu()).double()
    assert torch.isfinite(got).all()
    assert (got - ref).abs().max().item() < 2e-5


def test_qkv_attention_rejects_large_J(cuda):
    """Node counts without a fused tile (J not in 16 / 17 / 21 and J > 16, here the MANO J = 51)
    are refused; the caller runs the graph-linear + k_attention pair."""
    J, K, heads, B = 51, 192, 8, 8
    x = torch.zeros(B, J, K, device=cuda)
    W = torch.zeros(1, 3 * heads * 32, K, device=cuda)
    out = torch.zeros(B, J, heads * 32, device=cuda)
    g = torch.eye(J, device=cuda)
    nt = (ctypes.c_int64 * J)(*([0] * J))
    rc = _lib.lib().sd_test_qkv_attention(x.data_ptr(), K, W.data_ptr(), nt, g.data_ptr(), out.data_ptr(), B, J,
                                          heads, 1, 0, 0)
    assert rc < 0


LAYOUT_CASES = [  # (K1, K2, N, bias, film, act, res, rms, layout bits: x1 | x2 << 1 | res << 2 | out << 3)
    (192, 0, 192, True, True, 1, False, False, 0b1001),   # block1, blocked in/out
    (192, 0, 192, True, False, 1, True, False, 0b1101),   # block2 with blocked residual
    (256, 0, 192, False, False, 0, True, False, 0b1101),  # to_out
    (192, 192, 192, True, True, 1, False, False, 0b1011),  # final block1 on cat(x, r)
    (192, 0, 96, True, False, 0, False, False, 0b0001),   # final_glin: blocked in, row-major out
    (96, 96, 192, True, False, 0, False, False, 0b1000),   # init_lin: row-major in, blocked out
    (192, 0, 192, True, False, 1, True, False, 0b0101),   # mixed: blocked x / res, row-major out
]


@pytest.mark.parametrize("K1,K2,N,has_bias,has_film,act,has_res,rms,layout", LAYOUT_CASES)
@pytest.mark.parametrize("B", [64, 67])
def test_graph_linear_blocked_layout(K1, K2, N, has_bias, has_film, act, has_res, rms, layout, B, cuda):
    J, nty = 16, 10
    g = torch.Generator().manual_seed(K1 + K2 + N + layout + B)
    r = lambda *s: torch.rand(*s, generator=g) * 2 - 1  # noqa: E731
    x1, x2 = r(B, J, K1), (r(B, J, K2) if K2 else None)
    W = r(nty, N, K1 + K2) / (K1 + K2) ** 0.5
    types = torch.tensor([0, 1, 2, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 7, 8, 9])
    bias = r(nty, N) * 0.1 if has_bias else None
    ghat = F.normalize(torch.eye(J) + torch.rand(J, J, generator=g) * 0.1, p=1.0, dim=1)
    film = r(2 * N) * 0.5 if has_film else None
    res = r(B, J, N) if has_res else None
    ref = _gl_reference(x1, x2, W, bias, types, ghat, film, act, res, rms, 1)
    lay = lambda t, bit: None if t is None else (to_blocked(t) if layout & bit else t.contiguous())  # noqa: E731
    dev = lambda t: None if t is None else t.to(cuda)  # noqa: E731
    d = dict(x1=dev(lay(x1, 1)), x2=dev(lay(x2, 2)), res=dev(lay(res, 4)), W=dev(W), bias=dev(bias), ghat=dev(ghat),
             film=dev(film))
    n_out = to_blocked(torch.zeros(B, J, N)).numel() if layout & 8 else B * J * N
    out = torch.full((n_out,), float("nan"), device=cuda)
    nt = (ctypes.c_int64 * J)(*types.tolist())
    p = lambda a: None if a is None else a.data_ptr()  # noqa: E731
    _lib.check(_lib.lib().sd_test_graph_linear_layout(p(d["x1"]), K1, 1, p(d["x2"]), K2, p(d["W"]), p(d["bias"]), nt,
                                                      p(d["ghat"]), p(d["film"]), act, p(d["res"]), out.data_ptr(), B,
                                                      J, N, int(rms), layout, 0))
    torch.cuda.synchronize()
    got = from_blocked(out.cpu(), B, J, N) if layout & 8 else out.cpu().view(B, J, N)
    assert torch.isfinite(got).all()
    assert (got - ref).abs().max().item() < 2e-5

