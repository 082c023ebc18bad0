"""Transformer and RNN layers (reference: python/paddle/nn/layer/{transformer,rnn}.py)."""
from __future__ import annotations

import copy

import torch

from ...framework.tensor import Tensor
from .. import functional as F
from .common import Dropout, LayerList, LayerNorm, Linear
from .layers import Layer

_wrap = Tensor._wrap


class MultiHeadAttention(Layer):
    """paddle.nn.MultiHeadAttention; inputs [batch, seq, embed]. Uses the flash kernel when no mask."""

    def __init__(self, embed_dim, num_heads, dropout=0.0, kdim=None, vdim=None, need_weights=False,
                 weight_attr=None, bias_attr=None):
        super().__init__()
        self.embed_dim, self.num_heads = embed_dim, num_heads
        self.kdim, self.vdim = kdim or embed_dim, vdim or embed_dim
        self.head_dim = embed_dim // num_heads
        self.dropout, self.need_weights = dropout, need_weights
        self.q_proj = Linear(embed_dim, embed_dim, weight_attr, bias_attr)
        self.k_proj = Linear(self.kdim, embed_dim, weight_attr, bias_attr)
        self.v_proj = Linear(self.vdim, embed_dim, weight_attr, bias_attr)
        self.out_proj = Linear(embed_dim, embed_dim, weight_attr, bias_attr)

    def forward(self, query, key=None, value=None, attn_mask=None, cache=None):
        key = query if key is None else key
        value = query if value is None else value
        b, sq = query.shape[0], query.shape[1]
        q = self.q_proj(query)._t.reshape(b, sq, self.num_heads, self.head_dim)
        k = self.k_proj(key)._t.reshape(b, key.shape[1], self.num_heads, self.head_dim)
        v = self.v_proj(value)._t.reshape(b, value.shape[1], self.num_heads, self.head_dim)
        if attn_mask is None and not self.need_weights and (self.dropout == 0 or not self.training):
            out, _ = F.flash_attention(_wrap(q), _wrap(k), _wrap(v), 0.0, False, training=self.training)
            o = out._t
            w = None
        else:
            qt, kt, vt = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
            s = torch.matmul(qt, kt.transpose(-1, -2)) / (self.head_dim ** 0.5)
            if attn_mask is not None:
                m = attn_mask._t
                if m.dtype == torch.bool:
                    s = s.masked_fill(~m, float("-inf"))
                else:
                    s = s + m.to(s.dtype)
            w = torch.softmax(s, -1)
            if self.dropout and self.training:
                w = torch.nn.functional.dropout(w, self.dropout)
            o = torch.matmul(w, vt).transpose(1, 2)
        out = self.out_proj(_wrap(o.reshape(b, sq, self.embed_dim)))
        if self.need_weights:
            return out, _wrap(w)
        return out


def _get_act(name):
    return getattr(F, name)


class TransformerEncoderLayer(Layer):
    def __init__(self, d_model, nhead, dim_feedforward, dropout=0.1, activation="relu", attn_dropout=None,
                 act_dropout=None, normalize_before=False, weight_attr=None, bias_attr=None, layer_norm_eps=1e-5):
        super().__init__()
        attn_dropout = dropout if attn_dropout is None else attn_dropout
        act_dropout = dropout if act_dropout is None else act_dropout
        self.normalize_before = normalize_before
        self.self_attn = MultiHeadAttention(d_model, nhead, attn_dropout, weight_attr=weight_attr, bias_attr=bias_attr)
        self.linear1 = Linear(d_model, dim_feedforward, weight_attr, bias_attr)
        self.dropout = Dropout(act_dropout)
        self.linear2 = Linear(dim_feedforward, d_model, weight_attr, bias_attr)
        self.norm1 = LayerNorm(d_model, layer_norm_eps)
        self.norm2 = LayerNorm(d_model, layer_norm_eps)
        self.dropout1 = Dropout(dropout)
        self.dropout2 = Dropout(dropout)
        self.activation = _get_act(activation)

    def forward(self, src, src_mask=None, cache=None):
        res = src
        if self.normalize_before:
            src = self.norm1(src)
        src = res + self.dropout1(self.self_attn(src, src, src, src_mask))
        if not self.normalize_before:
            src = self.norm1(src)
        res = src
        if self.normalize_before:
            src = self.norm2(src)
        src = self.linear2(self.dropout(self.activation(self.linear1(src))))
        src = res + self.dropout2(src)
        if not self.normalize_before:
            src = self.norm2(src)
        return src


class TransformerEncoder(Layer):
    def __init__(self, encoder_layer, num_layers, norm=None):
        super().__init__()
        self.layers = LayerList([encoder_layer if i == 0 else copy.deepcopy(encoder_layer) for i in range(num_layers)])
        self.num_layers = num_layers
        self.norm = norm

    def forward(self, src, src_mask=None, cache=None):
        out = src
        for l in self.layers:
            out = l(out, src_mask)
        if self.norm is not None:
            out = self.norm(out)
        return out


class TransformerDecoderLayer(Layer):
    def __init__(self, d_model, nhead, dim_feedforward, dropout=0.1, activation="relu", attn_dropout=None,
                 act_dropout=None, normalize_before=False, weight_attr=None, bias_attr=None, layer_norm_eps=1e-5):
        super().__init__()
        attn_dropout = dropout if attn_dropout is None else attn_dropout
        act_dropout = dropout if act_dropout is None else act_dropout
        self.normalize_before = normalize_before
        self.self_attn = MultiHeadAttention(d_model, nhead, attn_dropout)
        self.cross_attn = MultiHeadAttention(d_model, nhead, attn_dropout)
        self.linear1 = Linear(d_model, dim_feedforward)
        self.dropout = Dropout(act_dropout)
        self.linear2 = Linear(dim_feedforward, d_model)
        self.norm1 = LayerNorm(d_model, layer_norm_eps)
        self.norm2 = LayerNorm(d_model, layer_norm_eps)
        self.norm3 = LayerNorm(d_model, layer_norm_eps)
        self.dropout1 = Dropout(dropout)
        self.dropout2 = Dropout(dropout)
        self.dropout3 = Dropout(dropout)
        self.activation = _get_act(activation)

    def forward(self, tgt, memory, tgt_mask=None, memory_mask=None, cache=None):
        res = tgt
        if self.normalize_before:
            tgt = self.norm1(tgt)
        tgt = res + self.dropout1(self.self_attn(tgt, tgt, tgt, tgt_mask))
        if not self.normalize_before:
            tgt = self.norm1(tgt)
        res = tgt
        if self.normalize_before:
            tgt = self.norm2(tgt)
        tgt = res + self.dropout2(self.cross_attn(tgt, memory, memory, memory_mask))
        if not self.normalize_before:
            tgt = self.norm2(tgt)
        res = tgt
        if self.normalize_before:
            tgt = self.norm3(tgt)
        tgt = res + self.dropout3(self.linear2(self.dropout(self.activation(self.linear1(tgt)))))
        if not self.normalize_before:
            tgt = self.norm3(tgt)
        return tgt


class TransformerDecoder(Layer):
    def __init__(self, decoder_layer, num_layers, norm=None):
        super().__init__()
        self.layers = LayerList([decoder_layer if i == 0 else copy.deepcopy(decoder_layer) for i in range(num_layers)])
        self.norm = norm

    def forward(self, tgt, memory, tgt_mask=None, memory_mask=None, cache=None):
        out = tgt
        for l in self.layers:
            out = l(out, memory, tgt_mask, memory_mask)
        if self.norm is not None:
            out = self.norm(out)
        return out


class Transformer(Layer):
    def __init__(self, d_model=512, nhead=8, num_encoder_layers=6, num_decoder_layers=6, dim_feedforward=2048,
                 dropout=0.1, activation="relu", attn_dropout=None, act_dropout=None, normalize_before=False,
                 weight_attr=None, bias_attr=None, custom_encoder=None, custom_decoder=None):
        super().__init__()
        enc = TransformerEncoderLayer(d_model, nhead, dim_feedforward, dropout, activation, attn_dropout, act_dropout,
                                      normalize_before)
        self.encoder = custom_encoder or TransformerEncoder(enc, num_encoder_layers,
                                                            LayerNorm(d_model) if normalize_before else None)
        dec = TransformerDecoderLayer(d_model, nhead, dim_feedforward, dropout, activation, attn_dropout, act_dropout,
                                      normalize_before)
        self.decoder = custom_decoder or TransformerDecoder(dec, num_decoder_layers,
                                                            LayerNorm(d_model) if normalize_before else None)

    def forward(self, src, tgt, src_mask=None, tgt_mask=None, memory_mask=None):
        mem = self.encoder(src, src_mask)
        return self.decoder(tgt, mem, tgt_mask, memory_mask)

    @staticmethod
    def generate_square_subsequent_mask(length):
        m = torch.triu(torch.full((length, length), float("-inf")), 1)
        from ...framework.place import current_torch_device

        return _wrap(m.to(current_torch_device()))


# ------------------------------------------------------------------ RNNs (MIOpen-backed through ATen)
class _RNNBase(Layer):
    _mode = "LSTM"

    def __init__(self, input_size, hidden_size, num_layers=1, direction="forward", time_major=False, dropout=0.0,
                 activation="tanh", weight_ih_attr=None, weight_hh_attr=None, bias_ih_attr=None, bias_hh_attr=None,
                 name=None):
        super().__init__()
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        self.time_major = time_major
        bidir = direction in ("bidirect", "bidirectional")
        self.num_directions = 2 if bidir else 1
        kw = dict(num_layers=num_layers, batch_first=not time_major, dropout=dropout, bidirectional=bidir)
        if self._mode == "LSTM":
            mod = torch.nn.LSTM(input_size, hidden_size, **kw)
        elif self._mode == "GRU":
            mod = torch.nn.GRU(input_size, hidden_size, **kw)
        else:
            mod = torch.nn.RNN(input_size, hidden_size, nonlinearity="relu" if activation == "relu" else "tanh", **kw)
        from ...framework.param import Parameter
        from ...framework.place import current_torch_device

        mod = mod.to(current_torch_device())
        self._names = []
        for n, p in mod.named_parameters():
            self.add_parameter(n, Parameter(p.data))
            self._names.append(n)
        object.__setattr__(self, "_mod", mod)

    def forward(self, inputs, initial_states=None, sequence_length=None):
        mod = self._mod
        params = {n: self._parameters[n]._t for n in self._names}
        hx = None
        if initial_states is not None:
            if isinstance(initial_states, (list, tuple)):
                hx = tuple(s._t for s in initial_states)
            else:
                hx = initial_states._t
        out, h = torch.func.functional_call(mod, params, (inputs._t, hx))
        if isinstance(h, tuple):
            return _wrap(out), tuple(_wrap(x) for x in h)
        return _wrap(out), _wrap(h)


class LSTM(_RNNBase):
    _mode = "LSTM"


class GRU(_RNNBase):
    _mode = "GRU"


class SimpleRNN(_RNNBase):
    _mode = "RNN"


from .rnn import RNNCellBase  # noqa: E402


class _CellBase(RNNCellBase):
    def __init__(self, input_size, hidden_size, mode, activation="tanh"):
        super().__init__()
        g = {"LSTM": 4, "GRU": 3, "RNN": 1}[mode]
        self.mode, self.hidden_size, self.activation = mode, hidden_size, activation
        self.input_size = input_size
        from .. import initializer as I

        k = 1.0 / hidden_size ** 0.5
        self.weight_ih = self.create_parameter([g * hidden_size, input_size], default_initializer=I.Uniform(-k, k))
        self.weight_hh = self.create_parameter([g * hidden_size, hidden_size], default_initializer=I.Uniform(-k, k))
        self.bias_ih = self.create_parameter([g * hidden_size], is_bias=True, default_initializer=I.Uniform(-k, k))
        self.bias_hh = self.create_parameter([g * hidden_size], is_bias=True, default_initializer=I.Uniform(-k, k))

    @property
    def state_shape(self):
        return ((self.hidden_size,), (self.hidden_size,)) if self.mode == "LSTM" else (self.hidden_size,)

    def forward(self, inputs, states=None):
        x = inputs._t
        b = x.shape[0]
        z = torch.zeros(b, self.hidden_size, device=x.device, dtype=x.dtype)
        if self.mode == "LSTM":
            h, c = (z, z) if states is None else (states[0]._t, states[1]._t)
            h2, c2 = torch._VF.lstm_cell(x, (h, c), self.weight_ih._t, self.weight_hh._t, self.bias_ih._t, self.bias_hh._t)
            return _wrap(h2), (_wrap(h2), _wrap(c2))
        h = z if states is None else states._t
        if self.mode == "GRU":
            h2 = torch._VF.gru_cell(x, h, self.weight_ih._t, self.weight_hh._t, self.bias_ih._t, self.bias_hh._t)
        else:
            fn = torch._VF.rnn_relu_cell if self.activation == "relu" else torch._VF.rnn_tanh_cell
            h2 = fn(x, h, self.weight_ih._t, self.weight_hh._t, self.bias_ih._t, self.bias_hh._t)
        return _wrap(h2), _wrap(h2)


class LSTMCell(_CellBase):
    def __init__(self, input_size, hidden_size, weight_ih_attr=None, weight_hh_attr=None, bias_ih_attr=None,
                 bias_hh_attr=None, proj_size=0, name=None):
        super().__init__(input_size, hidden_size, "LSTM")


class GRUCell(_CellBase):
    def __init__(self, input_size, hidden_size, weight_ih_attr=None, weight_hh_attr=None, bias_ih_attr=None,
                 bias_hh_attr=None, name=None):
        super().__init__(input_size, hidden_size, "GRU")


class SimpleRNNCell(_CellBase):
    def __init__(self, input_size, hidden_size, activation="tanh", weight_ih_attr=None, weight_hh_attr=None,
                 bias_ih_attr=None, bias_hh_attr=None, name=None):
        super().__init__(input_size, hidden_size, "RNN", activation)
