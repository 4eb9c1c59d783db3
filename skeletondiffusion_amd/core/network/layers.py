"""Denoiser building blocks with the reference's parameter layout.

Module / attribute names are fixed by the reference's state_dict (strict loading,
reference src/eval_prepare_model.py:72), so they match
src/core/network/layers/{graph_structural,attention}.py; the code itself is written for this
engine.  These modules serve `NonisotropicGaussianDiffusion.forward()` (training, autograd); on
the device every StaticGraphLinear runs forward and backward on the HIP training kernels
(training.py, sd_train.hip), the rest on torch ops.  Sampling never calls them: it runs on the
HIP engine (engine.py).
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F
from torch import nn
from torch.nn import Parameter, init

from ... import training as _training


class StaticGraphLinear(nn.Module):
    """Per-node-type linear map followed by graph mixing (graph_structural.py:30-43, 58-114).

    y[b, i] = sum_j Ghat[i, j] (W[type(j)] x[b, j] + bias[type(j)]),
    Ghat = G / rowsum|G| when `learn_influence`, else the fixed G (identity by default).
    """

    def __init__(self, in_features: int, out_features: int, *args, bias: bool = True,
                 num_nodes: Optional[int] = None, graph_influence=None, learn_influence: bool = False,
                 node_types: Optional[torch.Tensor] = None, weights_per_type: bool = False, **ignored):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.learn_influence = learn_influence
        if graph_influence is not None:
            assert num_nodes is None or num_nodes == graph_influence.shape[0], \
                "Number of Nodes or Graph Influence Matrix has to be given."
            num_nodes = graph_influence.shape[0]
            if isinstance(graph_influence, Parameter):
                assert learn_influence, "Graph Influence Matrix is a Parameter, therefore it must be learnable."
                self.G = graph_influence
            elif learn_influence:
                self.G = Parameter(graph_influence)
            else:
                self.register_buffer("G", graph_influence)
        else:
            assert num_nodes, "Number of Nodes or Graph Influence Matrix has to be given."
            eye = torch.eye(num_nodes, num_nodes)
            if learn_influence:
                self.G = Parameter(eye)
            else:
                self.register_buffer("G", eye)
        if weights_per_type and node_types is None:
            node_types = torch.arange(num_nodes)
        self.num_nodes = num_nodes
        if node_types is not None:
            node_types = torch.as_tensor(node_types, dtype=torch.long)
            lead = (int(node_types.max()) + 1,)
        else:
            lead = ()
        self.weight = Parameter(torch.empty(*lead, out_features, in_features))
        if bias:
            self.bias = Parameter(torch.empty(*lead, out_features))
        else:
            self.register_parameter("bias", None)
        self.node_type_index = node_types  # plain attribute, not a buffer (as the reference)
        self.reset_parameters()

    def reset_parameters(self) -> None:
        # same RNG consumption as the reference (graph_structural.py:17-28)
        init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.weight.dim() == 3:
            with torch.no_grad():
                self.weight[1:] = self.weight[0]
        if self.bias is not None:
            fan_in, _ = init._calculate_fan_in_and_fan_out(self.weight)
            bound = 1 / math.sqrt(fan_in)
            init.uniform_(self.bias, -bound, bound)

    def hip_ghat_ok(self) -> bool:
        G = self.G
        return (self.learn_influence and isinstance(G, torch.Tensor) and G.is_cuda and torch.is_grad_enabled()
                and G.dtype == torch.float32 and _training.hip_training_enabled() and G.dim() == 2
                and G.shape[0] == G.shape[1] <= _training.MAX_NODES)

    def ghat(self) -> torch.Tensor:
        if not self.learn_influence:
            return self.G
        pre = getattr(self, "_ghat_batched", None)
        if pre is not None:  # set by Denoiser.forward: every G normalised in one launch
            return pre
        G = self.G
        if (G.is_cuda and torch.is_grad_enabled() and G.dtype == torch.float32 and _training.hip_training_enabled()
                and G.dim() == 2 and G.shape[0] == G.shape[1] <= _training.MAX_NODES):
            # training on the device: one HIP launch each way (sd_train.hip k_l1norm_rows)
            return _training.l1norm_rows(G, 1e-12)
        return F.normalize(G, p=1.0, dim=1)

    def _hip_ok(self, x: torch.Tensor, g: torch.Tensor) -> bool:
        # the node-type validity check reads the (host) type vector: done once per (vector,
        # version, weight shape), not per call
        nt = self.node_type_index
        key = (id(nt), None if nt is None else nt._version, tuple(self.weight.shape), tuple(g.shape), x.shape[-2],
               x.dim())
        if getattr(self, "_hip_ok_key", None) != key:
            self._hip_ok_val = _training.hip_shapes_ok(x, self.weight, g, nt)
            self._hip_ok_key, self._hip_ok_src = key, nt  # the reference keeps id(nt) unique
        return self._hip_ok_val

    def _node_types_on(self, device: torch.device) -> Optional[torch.Tensor]:
        # device copy of the node-type vector, cached (one host-to-device copy, not one per call)
        nt = self.node_type_index
        if nt is None:
            return None
        key = (id(nt), nt._version, device)
        if getattr(self, "_nt_dev_key", None) != key:
            self._nt_dev = nt.to(device=device, dtype=torch.int64).contiguous()
            self._nt_dev_key, self._nt_dev_src = key, nt
        return self._nt_dev

    def forward(self, x: torch.Tensor, g: Optional[torch.Tensor] = None) -> torch.Tensor:
        g = self.ghat() if g is None else g
        if (x.is_cuda and torch.is_grad_enabled() and x.dtype == torch.float32
                and self.weight.dtype == torch.float32 and _training.hip_training_enabled()
                and self._hip_ok(x, g)):
            # training on the device: forward + backward on the HIP kernels (sd_train.hip)
            return _training.graph_linear(x, self.weight, self.bias, g, self._node_types_on(x.device))
        if self.node_type_index is not None:
            w = self.weight[self.node_type_index.to(self.weight.device)]       # (J, out, in)
            y = torch.einsum("noi,bni->bno", w, x)
            if self.bias is not None:
                y = y + self.bias[self.node_type_index.to(self.weight.device)]
        else:
            y = torch.matmul(x, self.weight.t())
            if self.bias is not None:
                y = y + self.bias
        return g.matmul(y)


class Residual(nn.Module):
    def __init__(self, fn):
        super().__init__()
        self.fn = fn

    def forward(self, x, *args, **kwargs):
        return self.fn(x, *args, **kwargs) + x


class RMSNorm(nn.Module):
    """x / max(||x||, 1e-12) * g * sqrt(dim)   (attention.py:30-36)."""

    def __init__(self, dim):
        super().__init__()
        self.g = Parameter(torch.ones(1, 1, dim))

    def forward(self, x):
        if (x.is_cuda and torch.is_grad_enabled() and x.dtype == torch.float32 and self.g.dtype == torch.float32
                and _training.hip_training_enabled() and x.shape[-1] <= 1024 and self.g.numel() == x.shape[-1]):
            # training on the device: forward + backward on HIP (sd_train.hip k_rmsnorm)
            return _training.rmsnorm(x, self.g, x.shape[-1] ** 0.5, 1e-12)
        return F.normalize(x, dim=-1) * self.g * (x.shape[-1] ** 0.5)


class NodeLayerNorm(nn.Module):
    """LayerNorm over the node axis (norm_type='layer', attention.py:19-28)."""

    def __init__(self, num_nodes):
        super().__init__()
        self.norm = nn.LayerNorm(num_nodes, elementwise_affine=True)

    def forward(self, x):
        return self.norm(x.transpose(-2, -1)).transpose(-2, -1)


class PreNorm(nn.Module):
    def __init__(self, dim, fn):
        super().__init__()
        self.fn = fn
        self.norm = RMSNorm(dim)

    def forward(self, x):
        return self.fn(self.norm(x))


class Block(nn.Module):
    """StaticGraphLinear -> (norm) -> FiLM -> tanh   (attention.py:49-75)."""

    def __init__(self, dim, dim_out, norm_type="none", act_type="tanh", **kwargs):
        super().__init__()
        self.proj = StaticGraphLinear(dim, dim_out, **kwargs)
        if norm_type == "none":
            self.norm = nn.Identity()
        elif norm_type == "layer":
            self.norm = NodeLayerNorm(kwargs["num_nodes"])
        else:
            raise AssertionError(f"Norm type {norm_type} not implemented!")
        if act_type != "tanh":
            raise AssertionError(f"Activation type {act_type} not implemented!")
        self.act = nn.Tanh()
        self.norm_type = norm_type

    def forward(self, x, scale_shift=None):
        x = self.norm(self.proj(x))
        if scale_shift is not None:
            scale, shift = scale_shift
            x = x * (scale + 1) + shift
        return self.act(x)


class ResnetBlock(nn.Module):
    """attention.py:78-102."""

    def __init__(self, dim, dim_out, *, time_emb_dim=None, groups=8, **kwargs):
        super().__init__()
        self.mlp = nn.Sequential(nn.Tanh(), nn.Linear(time_emb_dim, dim_out * 2)) \
            if time_emb_dim is not None else None
        self.block1 = Block(dim, dim_out, **kwargs)
        self.block2 = Block(dim_out, dim_out, **kwargs)
        self.res_linear = StaticGraphLinear(dim, dim_out, bias=False, **kwargs) \
            if dim != dim_out else nn.Identity()

    def forward(self, x, time_emb=None):
        scale_shift = None
        if self.mlp is not None and time_emb is not None:
            ss = self.mlp(time_emb).unsqueeze(1)
            if (ss.is_cuda and torch.is_grad_enabled() and ss.dtype == torch.float32 and x.dim() == 3
                    and _training.hip_training_enabled() and isinstance(self.block1.norm, nn.Identity)
                    and x.shape[0] <= 65535):
                # training on the device: block1's FiLM + tanh forward and backward on HIP
                y = self.block1.proj(x)
                if y.dtype == torch.float32:
                    h = self.block2(_training.film_tanh(y, ss))
                    return h + self.res_linear(x)
                scale_shift = ss.chunk(2, dim=-1)
                h = self.block2(self.block1.act(y * (scale_shift[0] + 1) + scale_shift[1]))
                return h + self.res_linear(x)
            scale_shift = ss.chunk(2, dim=-1)
        h = self.block2(self.block1(x, scale_shift=scale_shift))
        return h + self.res_linear(x)


class Attention(nn.Module):
    """Multi-head self-attention over the joint axis (attention.py:105-136)."""

    def __init__(self, dim, dim_out=None, heads=4, dim_head=32, qkv_bias: bool = False,
                 attn_dropout: float = 0.0, proj_dropout: float = 0.0, qk_norm: bool = False,
                 norm_layer=nn.Identity, **kwargs):
        super().__init__()
        self.scale = dim_head ** -0.5
        self.heads = heads
        self.dim_head = dim_head
        hidden = dim_head * heads
        dim_out = dim_out if dim_out is not None else dim
        self.to_qkv = StaticGraphLinear(dim, hidden * 3, bias=qkv_bias, **kwargs)
        self.to_out = StaticGraphLinear(hidden, dim_out, bias=False, **kwargs)
        self.attn_dropout = nn.Dropout(attn_dropout)
        self.out_dropout = nn.Dropout(proj_dropout)
        self.q_norm = norm_layer(dim_head) if qk_norm else nn.Identity()
        self.k_norm = norm_layer(dim_head) if qk_norm else nn.Identity()

    def forward(self, x):
        b, n, _ = x.shape
        qkv = self.to_qkv(x)
        if (qkv.is_cuda and torch.is_grad_enabled() and qkv.dtype == torch.float32 and _training.hip_training_enabled()
                and isinstance(self.q_norm, nn.Identity) and isinstance(self.k_norm, nn.Identity)
                and (not self.training or self.attn_dropout.p == 0.0) and 1 <= n <= 64 and 1 <= self.dim_head <= 64):
            # training on the device: the attention core forward + backward on HIP (sd_train.hip)
            out = _training.attention_core(qkv, self.heads, self.dim_head, self.scale)
            return self.out_dropout(self.to_out(out))
        q, k, v = (c.reshape(b, n, self.heads, self.dim_head).permute(0, 2, 3, 1)
                   for c in qkv.chunk(3, dim=-1))                       # (b, h, c, n)
        q, k = self.q_norm(q), self.k_norm(k)
        q = q * self.scale
        attn = torch.einsum("bhcn,bhcj->bhnj", q, k).softmax(dim=-1)
        attn = self.attn_dropout(attn)
        out = torch.einsum("bhnj,bhdj->bhnd", attn, v)
        out = out.permute(0, 2, 1, 3).reshape(b, n, self.heads * self.dim_head)
        return self.out_dropout(self.to_out(out))


class SinusoidalPosEmb(nn.Module):
    """denoising_diffusion_pytorch 1.9.4 SinusoidalPosEmb (restated; the package is not a
    dependency of this engine): emb = cat(sin(t f), cos(t f)), f_k = exp(-k ln(theta)/(half-1))."""

    def __init__(self, dim, theta=10000):
        super().__init__()
        self.dim = dim
        self.theta = theta

    def forward(self, x):
        half = self.dim // 2
        scale = math.log(self.theta) / (half - 1)
        freqs = torch.exp(torch.arange(half, device=x.device) * -scale)
        arg = x[:, None] * freqs[None, :]
        return torch.cat((arg.sin(), arg.cos()), dim=-1)


class RandomOrLearnedSinusoidalPosEmb(nn.Module):
    """denoising_diffusion_pytorch 1.9.4 learned / random Fourier features (restated)."""

    def __init__(self, dim, is_random=False):
        super().__init__()
        assert dim % 2 == 0
        self.weights = Parameter(torch.randn(dim // 2), requires_grad=not is_random)

    def forward(self, x):
        x = x[:, None]
        freqs = x * self.weights[None, :] * 2 * math.pi
        return torch.cat((x, freqs.sin(), freqs.cos()), dim=-1)
