"""Binding of the HIP graph-GRU decoder (`sd_gru_decode`, include/skeldiff.h) to the mirrored
`Decoder` module (core/network/autoencoder.py).  Tensors are passed by pointer on every call
(the decoder's weights are small and already on the device), so weight updates need no plan."""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import SkelDiffError, check


class DecoderEngine:
    def __init__(self, decoder, encoder=None, z_tanh: bool = True):
        self.dec = decoder
        self.enc = encoder
        self.z_tanh = z_tanh
        self._ws = None

    def _workspace(self, nbytes, dev):
        if self._ws is None or self._ws.numel() < nbytes or self._ws.device != dev:
            self._ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        return self._ws

    def encode(self, x: torch.Tensor) -> torch.Tensor:
        """z_activation(Encoder(x)) for x (B, T, J, F) -> (B, J, L) on the HIP encoder."""
        enc = self.enc
        if enc is None:
            raise SkelDiffError("no encoder bound")
        if enc.recurrent_arch != "StaticGraphGRU" or enc.num_layers != 1:
            raise SkelDiffError("the HIP encoder covers one StaticGraphGRU layer (the released configs)")
        if not (isinstance(enc.activation_fn, torch.nn.Tanh) and self.z_tanh):
            raise SkelDiffError("the HIP encoder covers encoder_act = z_activation = 'tanh' (the released configs)")
        cell = enc.rnn.layers[0]
        dev = cell.weight_hh.device
        if dev.type != "cuda":
            raise SkelDiffError("AutoEncoder.get_past_embedding runs on the MI355X HIP engine only: move the module "
                                "to a ROCm device first")
        keep = []

        def p(t):
            if t is None or not torch.is_tensor(t):
                return None
            t = t.detach().to(device=dev, dtype=torch.float32).contiguous()
            keep.append(t)
            return t.data_ptr()

        d = _lib.SDGruDecoderDesc()
        J = cell.num_nodes
        d.num_nodes, d.hidden_size, d.feature_size = J, cell.hidden_size, cell.input_size
        d.latent_size = enc.fc.out_features
        nt = cell.node_type_index
        if nt is not None:
            arr = (ctypes.c_int64 * J)(*[int(v) for v in nt.tolist()])
            keep.append(arr)
            d.num_node_types = int(cell.weight_hh.shape[0])
            d.node_types = ctypes.cast(arr, ctypes.POINTER(ctypes.c_int64))
        ih = enc.initial_hidden1
        d.init_G, d.init_weight, d.init_bias = p(ih.G), p(ih.weight), p(ih.bias)
        d.G, d.G_add = p(cell.G), None
        d.weight_ih, d.weight_hh, d.bias_ih, d.bias_hh = (p(cell.weight_ih), p(cell.weight_hh), p(cell.bias_ih),
                                                          p(cell.bias_hh))
        d.fc_G, d.fc_weight, d.fc_bias = p(enc.fc.G), p(enc.fc.weight), p(enc.fc.bias)
        B, T = x.shape[0], x.shape[1]
        if tuple(x.shape[2:]) != (J, d.feature_size):
            raise SkelDiffError(f"encode: x {tuple(x.shape)} is not (B, T, {J}, {d.feature_size})")
        x = x.detach().to(device=dev, dtype=torch.float32).contiguous()
        z = torch.empty((B, J, d.latent_size), device=dev, dtype=torch.float32)
        if B == 0:
            return z
        L_ = _lib.lib()
        nbytes = int(L_.sd_gru_encode_workspace_bytes(ctypes.byref(d), B, T))
        if nbytes == 0:
            raise SkelDiffError("sd_gru_encode_workspace_bytes: " + L_.sd_last_error().decode())
        ws = self._workspace(nbytes, dev)
        check(L_.sd_gru_encode(ctypes.byref(d), x.data_ptr(), B, T, z.data_ptr(), ws.data_ptr(), ws.numel(),
                               torch.cuda.current_stream(dev).cuda_stream))
        return z

    def _desc(self, keep):
        dec = self.dec
        if dec.recurrent_arch != "StaticGraphGRU" or dec.num_layers != 1:
            raise SkelDiffError("the HIP decoder covers one StaticGraphGRU layer (the released configs)")
        cell = dec.rnn.layers[0]
        dev = cell.weight_hh.device
        if dev.type != "cuda":
            raise SkelDiffError("AutoEncoder.decode runs on the MI355X HIP engine only: move the module to a ROCm "
                                "device first; there is no CPU decoding path")
        if cell.clockwork:
            raise SkelDiffError("clockwork GRU cells are not supported by the HIP decoder")

        def p(t):
            if t is None or not torch.is_tensor(t):
                return None
            t = t.detach().to(device=dev, dtype=torch.float32).contiguous()
            keep.append(t)
            return t.data_ptr()

        d = _lib.SDGruDecoderDesc()
        J = cell.num_nodes
        d.num_nodes, d.hidden_size = J, cell.hidden_size
        d.feature_size = dec.fc.out_features
        d.latent_size = cell.input_size - d.feature_size
        nt = cell.node_type_index
        if nt is not None:
            arr = (ctypes.c_int64 * J)(*[int(v) for v in nt.tolist()])
            keep.append(arr)
            d.num_node_types = int(cell.weight_hh.shape[0])
            d.node_types = ctypes.cast(arr, ctypes.POINTER(ctypes.c_int64))
        else:
            d.num_node_types = 0
        ih, fc = dec.initial_hidden_h, dec.fc
        d.init_G, d.init_weight, d.init_bias = p(ih.G), p(ih.weight), p(ih.bias)
        d.G = p(cell.G)
        d.G_add = p(cell.G_add)
        d.weight_ih, d.weight_hh = p(cell.weight_ih), p(cell.weight_hh)
        d.bias_ih, d.bias_hh = p(cell.bias_ih), p(cell.bias_hh)
        d.fc_G, d.fc_weight, d.fc_bias = p(fc.G), p(fc.weight), p(fc.bias)
        if not (ih.learn_influence and fc.learn_influence and cell.learn_influence):
            raise SkelDiffError("the HIP decoder expects learn_influence=True graph layers (decoder.py:32-57)")
        return d, dev

    def decode(self, x2: torch.Tensor, h: torch.Tensor, ph: int) -> torch.Tensor:
        """x2 (B, 2, J, F) = the last two observed frames, h (B, J, L) -> (B, ph, J, F)."""
        keep = []
        d, dev = self._desc(keep)
        B, J, F, L = h.shape[0], d.num_nodes, d.feature_size, d.latent_size
        if tuple(x2.shape[1:]) != (2, J, F) or tuple(h.shape[1:]) != (J, L) or x2.shape[0] != B:
            raise SkelDiffError(f"decode: x {tuple(x2.shape)} / h {tuple(h.shape)} do not match (B, 2, {J}, {F}) / "
                                f"(B, {J}, {L})")
        x2 = x2.detach().to(device=dev, dtype=torch.float32).contiguous()
        h = h.detach().to(device=dev, dtype=torch.float32).contiguous()
        out = torch.empty((B, ph, J, F), device=dev, dtype=torch.float32)
        if B == 0:
            return out
        L_ = _lib.lib()
        nbytes = int(L_.sd_gru_decode_workspace_bytes(ctypes.byref(d), B, ph))
        if nbytes == 0:
            raise SkelDiffError("sd_gru_decode_workspace_bytes: " + L_.sd_last_error().decode())
        ws = self._workspace(nbytes, dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        check(L_.sd_gru_decode(ctypes.byref(d), x2.data_ptr(), h.data_ptr(), B, int(ph), out.data_ptr(),
                               ws.data_ptr(), ws.numel(), stream))
        return out
