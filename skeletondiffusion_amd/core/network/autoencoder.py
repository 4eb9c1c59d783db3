"""Mirror of the reference's motion autoencoder (SURVEY.md §8f "next" #1): the graph-GRU
`Encoder` that turns the observed past into the conditioning latent, and the `Decoder` that
unrolls the sampled latent into `ph` future frames (`src/core/network/nn/{autoencoder,encoder,
decoder}.py`, `src/core/network/layers/recurrent.py:208-401`).  Same constructor kwargs and
state_dict keys as the reference, so its autoencoder checkpoints load strictly.

`AutoEncoder.decode` -- the step after `sample()` in the evaluation (`eval_prepare_model.py:
106-116`), run on bs x 50 rows for ph frames -- goes to the HIP decoder (`sd_gru_decode`) and
`get_past_embedding` (the conditioning latents) to the HIP encoder (`sd_gru_encode`) when the
module lives on a ROCm device; on the CPU they raise (no CPU evaluation path).  `forward` /
`autoencode` (training, autograd) stay torch ops.
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.nn import Parameter

from .layers import StaticGraphLinear

__all__ = ["StaticGraphGRUCell", "StaticGraphGRU", "Encoder", "Decoder", "AutoEncoder"]


def _gmm(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """graph_structural.py:7-8: per-node x[b, n] @ w[n] (w: (n, in, out))."""
    return torch.einsum("ndo,bnd->bno", w, x)


class StaticGraphGRUCell(nn.Module):
    """recurrent.py:208-366 (the GRU cell; clockwork off -> the update mask is 1)."""

    def __init__(self, input_size: int, hidden_size: int, num_nodes: Optional[int] = None, dropout: float = 0.,
                 recurrent_dropout: float = 0., graph_influence=None, learn_influence: bool = False,
                 additive_graph_influence=None, learn_additive_graph_influence: bool = False,
                 node_types: Optional[torch.Tensor] = None, weights_per_type: bool = False,
                 clockwork: bool = False, bias: bool = True):
        super().__init__()
        self.input_size, self.hidden_size = input_size, hidden_size
        self.learn_influence = learn_influence
        self.learn_additive_graph_influence = learn_additive_graph_influence
        if graph_influence is not None:
            num_nodes = graph_influence.shape[0]
            if isinstance(graph_influence, Parameter) or learn_influence:
                self.G = graph_influence if isinstance(graph_influence, Parameter) else Parameter(graph_influence)
            else:
                self.register_buffer("G", graph_influence)
        else:
            assert num_nodes, "Number of Nodes or Graph Influence Matrix has to be given."
            eye = torch.eye(num_nodes, num_nodes)
            if learn_influence:
                self.G = Parameter(eye)
            else:
                self.register_buffer("G", eye)
        if additive_graph_influence is not None:
            if isinstance(additive_graph_influence, Parameter) or learn_additive_graph_influence:
                self.G_add = (additive_graph_influence if isinstance(additive_graph_influence, Parameter)
                              else Parameter(additive_graph_influence))
            else:
                self.register_buffer("G_add", additive_graph_influence)
        elif learn_additive_graph_influence:
            self.G_add = Parameter(torch.zeros_like(self.G))
        else:
            self.G_add = 0.
        if weights_per_type and node_types is None:
            node_types = torch.arange(num_nodes)
        if node_types is not None:
            node_types = torch.as_tensor(node_types, dtype=torch.long)
            nt = int(node_types.max()) + 1
            self.weight_ih = Parameter(torch.empty(nt, 3 * hidden_size, input_size))
            self.weight_hh = Parameter(torch.empty(nt, 3 * hidden_size, hidden_size))
            self.register_buffer("node_type_index", node_types)
            lead = (nt,)
        else:
            self.weight_ih = Parameter(torch.empty(3 * hidden_size, input_size))
            self.weight_hh = Parameter(torch.empty(3 * hidden_size, hidden_size))
            self.register_buffer("node_type_index", None)
            lead = ()
        if bias:
            self.bias_ih = Parameter(torch.empty(*lead, 3 * hidden_size))
            self.bias_hh = Parameter(torch.empty(*lead, 3 * hidden_size))
        else:
            self.bias_ih = self.bias_hh = None
        self.clockwork = clockwork
        if clockwork:
            phase = torch.arange(0., hidden_size)
            phase = torch.floor((phase - phase.min()) / phase.max() * 8. + 1.)
        else:
            phase = torch.ones(hidden_size)
        self.register_buffer("phase", phase)
        self.dropout = nn.Dropout(dropout)
        self.r_dropout = nn.Dropout(recurrent_dropout)
        self.num_nodes = num_nodes
        stdv = 1.0 / math.sqrt(hidden_size)  # recurrent.py:310-318
        for w in self.parameters():
            if w is self.G or w is self.G_add:
                continue
            w.data.uniform_(-stdv, stdv)

    def _typed(self, w):
        return w[self.node_type_index] if self.node_type_index is not None else w

    def forward(self, input: torch.Tensor, state, t: int = 0):
        hx, gx = state
        if hx is None:
            hx = input.new_zeros(input.shape[0], self.num_nodes, self.hidden_size)
        if gx is None:
            gx = F.normalize(self.G, p=1., dim=1) if self.learn_influence else self.G
        hx = self.r_dropout(hx)
        w_ih, w_hh = self._typed(self.weight_ih), self._typed(self.weight_hh)
        b_ih = self._typed(self.bias_ih) if self.bias_ih is not None else 0.
        b_hh = self._typed(self.bias_hh) if self.bias_hh is not None else 0.
        mm = _gmm if self.node_type_index is not None else torch.matmul
        c_mask = (torch.remainder(torch.tensor(t + 1., device=input.device), self.phase) < 0.01).type_as(hx)
        x_res = torch.matmul(gx, self.dropout(mm(input, w_ih.transpose(-2, -1))) + b_ih)
        h_res = torch.matmul(gx, mm(hx, w_hh.transpose(-2, -1)) + b_hh)
        i_r, i_z, i_n = x_res.chunk(3, 2)
        h_r, h_z, h_n = h_res.chunk(3, 2)
        r = torch.sigmoid(i_r + h_r)
        z = torch.sigmoid(i_z + h_z)
        n = torch.tanh(i_n + r * h_n)
        hy = n - n * z + z * hx
        hy = c_mask * hy + (1 - c_mask) * hx
        gx = gx + self.G_add
        if self.learn_influence or self.learn_additive_graph_influence:
            gx = F.normalize(gx, p=1., dim=1)
        return hy, (hy, gx)


class StaticGraphGRU(nn.Module):
    """recurrent.py:369-391: stacked cells over the time axis of (B, T, N, D) inputs."""

    def __init__(self, input_size: int, hidden_size: int, num_layers: int = 1, layer_dropout: float = 0.0, **kwargs):
        super().__init__()
        self.layers = nn.ModuleList([StaticGraphGRUCell(input_size, hidden_size, **kwargs)] +
                                    [StaticGraphGRUCell(hidden_size, hidden_size, **kwargs)
                                     for _ in range(num_layers - 1)])
        self.dropout = nn.Dropout(layer_dropout)

    def forward(self, input: torch.Tensor, states: Optional[List] = None, t_i: int = 0):
        if states is None:
            states = [(None, None)] * len(self.layers)
        output_states = []
        output = input
        for i, layer in enumerate(self.layers):
            state = states[i]
            outs = []
            for t, x in enumerate(output.unbind(1)):
                out, state = layer(x, state, t_i + t)
                outs.append(out)
            output = self.dropout(torch.stack(outs, dim=1))
            output_states.append(state)
        return output, output_states


def _recurrent(arch: str):
    if arch != "StaticGraphGRU":
        raise NotImplementedError(f"recurrent arch {arch!r}: only StaticGraphGRU (the released configs) is built")
    return StaticGraphGRU


class Encoder(nn.Module):
    """encoder.py:10-81: GRU over the observed frames, then tanh(fc(last hidden))."""

    def __init__(self, num_nodes: int, input_size: int, hidden_size: int, output_size: int,
                 node_types: Optional[torch.Tensor] = None, enc_num_layers: int = 1, dropout: float = 0.,
                 encoder_act: str = "tanh", recurrent_arch: str = "StaticGraphGRU", **kwargs):
        super().__init__()
        assert encoder_act in ("tanh", "identity"), "not implemented"
        self.activation_fn = nn.Tanh() if encoder_act == "tanh" else nn.Identity()
        self.num_layers = enc_num_layers
        self.recurrent_arch = recurrent_arch
        self.rnn = _recurrent(recurrent_arch)(input_size, hidden_size, num_layers=enc_num_layers,
                                              node_types=node_types, num_nodes=num_nodes, bias=True,
                                              clockwork=False, learn_influence=True)
        self.fc = StaticGraphLinear(hidden_size, output_size, num_nodes=num_nodes, node_types=node_types,
                                    bias=True, learn_influence=True)
        self.initial_hidden1 = StaticGraphLinear(input_size, hidden_size, num_nodes=num_nodes,
                                                 node_types=node_types, bias=True, learn_influence=True)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x: torch.Tensor, state=None):
        if state is None:
            state = [(self.initial_hidden1(x[:, 0]), None)] * self.num_layers
        y, state = self.rnn(input=x, states=state)
        return self.activation_fn(self.fc(self.dropout(y[:, -1]))), state


class Decoder(nn.Module):
    """decoder.py:9-104: GRU unrolled for ph frames from [last frame, latent], tanh(fc(h))."""

    def __init__(self, num_nodes: int, feature_size: int, input_size: int, hidden_size: int, output_size: int,
                 node_types: Optional[torch.Tensor] = None, dec_num_layers: int = 1, dropout: float = 0.,
                 param_groups=None, recurrent_arch_decoder: str = "StaticGraphGRU", **kwargs):
        super().__init__()
        self.param_groups = param_groups
        self.num_layers = dec_num_layers
        self.if_consider_hip = kwargs["if_consider_hip"]
        self.activation_fn = nn.Tanh()
        self.recurrent_arch = recurrent_arch_decoder
        self.rnn = _recurrent(recurrent_arch_decoder)(feature_size + input_size, hidden_size, num_nodes=num_nodes,
                                                      num_layers=dec_num_layers, learn_influence=True,
                                                      node_types=node_types, recurrent_dropout=dropout,
                                                      learn_additive_graph_influence=True, clockwork=False)
        self.initial_hidden_h = StaticGraphLinear(feature_size + input_size, hidden_size, num_nodes=num_nodes,
                                                  learn_influence=True, node_types=node_types)
        self.fc = StaticGraphLinear(hidden_size, output_size, num_nodes=num_nodes, learn_influence=True,
                                    node_types=node_types)
        self.dropout = nn.Dropout(dropout)

    def init_recurrent_hidden(self, x, h, z, state=None):
        x_t = x[:, -1]
        x_t_1 = x[:, -2] if state is None else state
        rnn_h = self.initial_hidden_h(torch.cat([x_t_1, h], dim=-1))
        return torch.cat([x_t, h], dim=-1).unsqueeze(1), [(rnn_h, None)] * self.num_layers

    def forward(self, x: torch.Tensor, h: torch.Tensor, z: torch.Tensor, ph: int = 1, state=None):
        """Torch forward (training / autograd); `AutoEncoder.decode` uses the HIP decoder."""
        x_t_s = x[:, -1].clone()
        rec_input, hidden = self.init_recurrent_hidden(x=x, h=h, z=z, state=state)
        out = []
        for i in range(ph):
            rnn_out, hidden = self.rnn(input=rec_input, states=hidden, t_i=i)
            out.append(self.activation_fn(self.fc(self.dropout(rnn_out.squeeze(1)))))
        return torch.stack(out, dim=1), x_t_s


class AutoEncoder(nn.Module):
    """autoencoder.py:8-102."""

    def __init__(self, num_nodes: int, encoder_hidden_size: int, decoder_hidden_size: int, latent_size: int,
                 node_types: Optional[torch.Tensor] = None, input_size: int = 3, z_activation: str = "tanh",
                 enc_num_layers: int = 1, loss_pose_type: str = "l1", **kwargs):
        super().__init__()
        self.param_groups = [{}]
        self.latent_size = latent_size
        self.loss_pose_type = loss_pose_type
        self.encoder = Encoder(num_nodes=num_nodes, input_size=input_size, hidden_size=encoder_hidden_size,
                               output_size=latent_size, node_types=node_types, enc_num_layers=enc_num_layers,
                               recurrent_arch=kwargs["recurrent_arch_enc"])
        assert kwargs["output_size"] == input_size
        self.decoder = Decoder(num_nodes=num_nodes, input_size=latent_size, feature_size=input_size,
                               hidden_size=decoder_hidden_size, node_types=node_types,
                               param_groups=self.param_groups, **kwargs)
        assert z_activation in ["tanh", "identity"], \
            f"z_activation must be either 'tanh' or 'identity', but got {z_activation}"
        self.z_activation = nn.Tanh() if z_activation == "tanh" else nn.Identity()
        self._engine = None

    def forward(self, x):
        h, _ = self.encoder(x)
        return h

    def _hip(self):
        from ... import decoder_engine

        if self._engine is None:
            self._engine = decoder_engine.DecoderEngine(self.decoder, self.encoder,
                                                        z_tanh=isinstance(self.z_activation, nn.Tanh))
        return self._engine

    def get_past_embedding(self, past, state=None):
        """z_activation(encoder(past)) on the HIP encoder (the conditioning latents of sample(),
        eval_prepare_model.py:89-99); no_grad as the reference."""
        if state is not None:
            raise NotImplementedError("get_past_embedding(state=...) is not used by the evaluation and not built")
        return self._hip().encode(past)

    def get_embedding(self, future, state=None):
        return self.forward(future)

    def get_train_embeddings(self, y, past, state=None):
        return self.get_past_embedding(past, state=state), self.get_embedding(y, state=state)

    def decode(self, x: torch.Tensor, h: torch.Tensor, z: torch.Tensor, ph: int = 1, state=None):
        """(B, T_obs, J, F) past, (B, J, latent) sampled latent -> (B, ph, J, F) on the HIP decoder
        (decoder.py:85-104 semantics; `z` is unused there too)."""
        if state is not None:
            raise NotImplementedError("decode(state=...) is not used by the evaluation and not built")
        return self._hip().decode(x[:, -2:], h, ph)

    def autoencode(self, y, past, ph=1, state=None):
        """Training-time reconstruction on torch ops (autograd)."""
        with torch.no_grad():
            z_past = self.z_activation(self(past))
        z = self.get_embedding(y, state=state)
        out, _ = self.decoder(x=past[:, -2:], h=z, z=z_past, ph=ph, state=state)
        return out, z_past, z

    def loss(self, y_pred, y, type=None, reduction="mean", **kwargs):
        type = self.loss_pose_type if type is None else type
        if type == "mse":
            out = nn.MSELoss(reduction="none")(y_pred, y)
        elif type in ["l1", "L1"]:
            out = nn.L1Loss(reduction="none")(y_pred, y)
        else:
            assert 0, "Not implemnted"
        loss = out.sum(-1).mean(-1).mean(-1)
        if reduction == "mean":
            return loss.mean()
        if reduction == "none":
            return loss
        assert 0, "Not implemnted"
