"""Cell-driven recurrent wrappers: RNNCellBase, RNN, BiRNN and the functional rnn / birnn
(reference: python/paddle/nn/layer/rnn.py — RNNCellBase :210, RNN :1339, BiRNN :1431,
_rnn_dynamic_graph :176).

The fused multi-layer LSTM / GRU / SimpleRNN layers (layer/transformer.py) run MIOpen's fused RNN
through ATen; these wrappers drive ANY cell (the built-in cells or a user RNNCellBase subclass) step
by step with the reference semantics: batch-major inputs unless ``time_major``, ``sequence_length``
freezes a sequence's state after its last valid step (outputs of padded steps are still produced),
``is_reverse`` runs right-to-left, and states may be nested tuples (LSTM's (h, c)).
"""
from __future__ import annotations

import torch

from ...framework.tensor import Tensor
from .layers import Layer

_wrap = Tensor._wrap


def _t(x):
    return x._t if isinstance(x, Tensor) else x


def _map(fn, *structs):
    s0 = structs[0]
    if isinstance(s0, (tuple, list)):
        return type(s0)(_map(fn, *parts) for parts in zip(*structs))
    return fn(*structs)


class RNNCellBase(Layer):
    """Base of recurrent cells: ``forward(inputs, states) -> (outputs, new_states)`` plus the initial
    state helpers the RNN wrappers use."""

    def get_initial_states(self, batch_ref, shape=None, dtype=None, init_value=0.0, batch_dim_idx=0):
        ref = _t(batch_ref[0] if isinstance(batch_ref, (tuple, list)) else batch_ref)
        b = ref.shape[batch_dim_idx]
        shape = self.state_shape if shape is None else shape
        dt = ref.dtype if dtype is None else dtype
        if isinstance(dt, str):
            from ...framework.dtype import convert_dtype

            dt = convert_dtype(dt)

        def mk(shp):
            shp = [shp] if isinstance(shp, int) else list(shp)
            return _wrap(torch.full([b] + shp, float(init_value), dtype=dt, device=ref.device))

        if isinstance(shape, (tuple, list)) and shape and isinstance(shape[0], (tuple, list)):
            return tuple(mk(s) for s in shape)
        return mk(shape)

    @property
    def state_shape(self):
        raise NotImplementedError("RNNCellBase subclasses define state_shape")

    @property
    def state_dtype(self):
        return None


def rnn(cell, inputs, initial_states=None, sequence_length=None, time_major=False, is_reverse=False, **kwargs):
    """Run ``cell`` over the time axis (reference nn/layer/rnn.py:176).  -> (outputs, final_states)."""
    x0 = _t(inputs[0] if isinstance(inputs, (tuple, list)) else inputs)
    tdim = 0 if time_major else 1
    T = x0.shape[tdim]
    if initial_states is None:
        initial_states = cell.get_initial_states(batch_ref=inputs, batch_dim_idx=1 if time_major else 0)
    seq = _map(lambda a: _t(a) if time_major else _t(a).transpose(0, 1), inputs)  # [T, B, ...]
    mask = None
    if sequence_length is not None:
        lens = _t(sequence_length).to(x0.device)
        mask = (torch.arange(T, device=x0.device)[:, None] < lens[None, :])  # [T, B]
    order = range(T - 1, -1, -1) if is_reverse else range(T)
    states = initial_states
    outs = [None] * T
    for i in order:
        step_in = _map(lambda a: _wrap(a[i]), seq)
        out, new_states = cell(step_in, states, **kwargs)
        if mask is not None:
            m = mask[i]

            def keep(old, new, m=m):
                o, n = _t(old), _t(new)
                mm = m.reshape([-1] + [1] * (n.dim() - 1)).to(n.dtype)
                return _wrap(n * mm + o * (1 - mm))

            new_states = _map(keep, states, new_states)
        states = new_states
        outs[i] = out
    stacked = _map(lambda *steps: torch.stack([_t(s) for s in steps], 0), *outs)
    final_out = _map(lambda o: _wrap(o if time_major else o.transpose(0, 1)), stacked)
    return final_out, states


def birnn(cell_fw, cell_bw, inputs, initial_states=None, sequence_length=None, time_major=False, **kwargs):
    """Forward and reverse passes, outputs concatenated on the feature axis (reference :281)."""
    if initial_states is None:
        s_fw = s_bw = None
    else:
        s_fw, s_bw = initial_states
    o_fw, st_fw = rnn(cell_fw, inputs, s_fw, sequence_length, time_major, False, **kwargs)
    o_bw, st_bw = rnn(cell_bw, inputs, s_bw, sequence_length, time_major, True, **kwargs)
    out = _map(lambda a, b: _wrap(torch.cat([_t(a), _t(b)], -1)), o_fw, o_bw)
    return out, (st_fw, st_bw)


class RNN(Layer):
    """Wrap a cell into a sequence layer (reference RNN :1339)."""

    def __init__(self, cell, is_reverse=False, time_major=False):
        super().__init__()
        self.cell = cell
        if not hasattr(cell, "call"):
            self.cell.call = cell.forward
        self.is_reverse = is_reverse
        self.time_major = time_major

    def forward(self, inputs, initial_states=None, sequence_length=None, **kwargs):
        return rnn(self.cell, inputs, initial_states, sequence_length, self.time_major, self.is_reverse, **kwargs)


class BiRNN(Layer):
    """Bidirectional wrapper of two cells (reference BiRNN :1431)."""

    def __init__(self, cell_fw, cell_bw, time_major=False):
        super().__init__()
        self.cell_fw = cell_fw
        self.cell_bw = cell_bw
        if cell_fw.input_size != cell_bw.input_size:
            raise ValueError("BiRNN: cell_fw and cell_bw must take the same input size")
        self.time_major = time_major

    def forward(self, inputs, initial_states=None, sequence_length=None, **kwargs):
        if isinstance(initial_states, (list, tuple)) and len(initial_states) != 2:
            raise ValueError("BiRNN: initial_states must be (states_fw, states_bw)")
        return birnn(self.cell_fw, self.cell_bw, inputs, initial_states, sequence_length, self.time_major, **kwargs)
