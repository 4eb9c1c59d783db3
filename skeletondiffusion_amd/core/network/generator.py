"""The SkeletonDiffusion Denoiser with the reference constructor and parameter layout
(reference src/core/network/nn/generator.py:8-107).

`forward` is the torch (autograd) path used by training.  Sampling reads this module's
parameters into a HIP plan (skeletondiffusion_amd/engine.py) and never calls `forward`.
"""
from __future__ import annotations

import torch
from torch import nn

from ... import training as _training
from .layers import (Attention, PreNorm, RandomOrLearnedSinusoidalPosEmb, Residual, ResnetBlock,
                     SinusoidalPosEmb, StaticGraphLinear)


class Denoiser(nn.Module):
    def __init__(self, dim, out_dim, channels: int, cond_dim: int = 0, depth=1, self_condition=False,
                 resnet_block_groups=8, learned_variance=False, learned_sinusoidal_cond=False,
                 random_fourier_features=False, learned_sinusoidal_dim=16,
                 sinusoidal_pos_emb_theta=10000, attn_dim_head=32, attn_heads=4, use_attention=True,
                 **kwargs):
        super().__init__()
        self.channels = channels
        self.self_condition = self_condition
        # engine-facing configuration
        self.dim, self.cond_dim, self.depth = dim, cond_dim, depth
        self.attn_heads, self.attn_dim_head, self.use_attention = attn_heads, attn_dim_head, use_attention
        self.learned_variance = learned_variance
        self.sinusoidal_pos_emb_theta = sinusoidal_pos_emb_theta
        self.learned_time_embedding = bool(learned_sinusoidal_cond or random_fourier_features)
        self.graph_kwargs = dict(kwargs)

        width = dim + cond_dim                                   # "diffusion_size"
        in_width = dim * (2 if self_condition else 1) + cond_dim
        self.init_lin = StaticGraphLinear(in_width, width, bias=True, **kwargs)

        time_dim = width * 4
        if self.learned_time_embedding:
            pos = RandomOrLearnedSinusoidalPosEmb(learned_sinusoidal_dim, random_fourier_features)
            fourier_dim = learned_sinusoidal_dim + 1
        else:
            pos = SinusoidalPosEmb(width, theta=sinusoidal_pos_emb_theta)
            fourier_dim = width
        self.time_mlp = nn.Sequential(pos, nn.Linear(fourier_dim, time_dim), nn.GELU(),
                                      nn.Linear(time_dim, time_dim))

        def res_block(d_in):
            return ResnetBlock(d_in, width, time_emb_dim=time_dim, groups=resnet_block_groups, **kwargs)

        def mixer():
            if use_attention:
                inner = Attention(width, heads=attn_heads, dim_head=attn_dim_head, **kwargs)
            else:
                inner = StaticGraphLinear(width, width, bias=False, **kwargs)
            return Residual(PreNorm(width, inner))

        # 2*depth (ResnetBlock, mixer) pairs; the very last mixer is an Identity (generator.py:58-77)
        self.layers = nn.ModuleList([])
        for i in range(depth):
            self.layers.append(nn.ModuleList([res_block(width), mixer()]))
            self.layers.append(nn.ModuleList([res_block(width),
                                              mixer() if i != depth - 1 else nn.Identity()]))

        self.out_dim = out_dim * (2 if learned_variance else 1)
        self.final_res_block = res_block(2 * width)
        self.final_glin = StaticGraphLinear(width, self.out_dim, bias=True, **kwargs)

    @property
    def node_types(self):
        return self.init_lin.node_type_index

    @property
    def learn_influence(self):
        return self.init_lin.learn_influence

    def forward(self, x, time, x_self_cond=None, x_cond=None):
        # training on the device: all learnable G-hat of the graph-linears normalised in one HIP
        # launch each way (training.l1norm_rows_many) instead of one per layer call
        gls = [m for m in self.modules() if isinstance(m, StaticGraphLinear) and m.hip_ghat_ok()]
        if len(gls) > 1 and len({tuple(m.G.shape) for m in gls}) == 1 and len({m.G.device for m in gls}) == 1:
            for m, gh in zip(gls, _training.l1norm_rows_many([m.G for m in gls], 1e-12)):
                m._ghat_batched = gh
            try:
                return self._forward(x, time, x_self_cond, x_cond)
            finally:
                for m in gls:
                    m._ghat_batched = None
        return self._forward(x, time, x_self_cond, x_cond)

    def _forward(self, x, time, x_self_cond=None, x_cond=None):
        if self.self_condition:
            x_self_cond = x_self_cond if x_self_cond is not None else torch.zeros_like(x)
            x = torch.cat((x_self_cond, x), dim=-1)
        if x_cond is not None:
            x = torch.cat([x_cond, x], dim=-1)
        x = self.init_lin(x)
        r = x.clone()
        t = self.time_mlp(time)
        for block, mixer in self.layers:
            x = mixer(block(x, t))
        x = self.final_res_block(torch.cat((x, r), dim=-1), t)
        return self.final_glin(x)
