"""paddle.quantization.quanters (reference: python/paddle/quantization/quanters/abs_max.py).

FakeQuanterWithAbsMaxObserver: QAT fake quantization with a moving-average abs-max scale
(scale = accum / state, accum = rate * accum + max|x|, state = rate * state + 1) and a straight-through gradient.
"""
from __future__ import annotations

import torch

from ..framework.tensor import Tensor
from .base_quanter import BaseQuanter
from .factory import QuanterFactory

_w = Tensor._wrap


def _t(x):
    return x._t if isinstance(x, Tensor) else x


class FakeQuanterWithAbsMaxObserverLayer(BaseQuanter):
    """Moving-average abs-max fake quanter: scale = accum/state, accum = rate*accum + max|x|."""

    def __init__(self, layer, name=None, moving_rate=0.9, bit_length=8, dtype="float32"):
        super().__init__()
        self._moving_rate, self._bit_length = moving_rate, bit_length
        self.register_buffer("_scale", _w(torch.full((1,), 1e-3)))
        self.register_buffer("_state", _w(torch.zeros(1)))
        self.register_buffer("_accum", _w(torch.zeros(1)))

    def forward(self, input):
        from ..nn.quant.quant_layers import fake_quant_dequant

        x = _t(input)
        if self.training:
            with torch.no_grad():
                cur = x.detach().abs().max().float().reshape(1).to(self._accum._t.device)
                self._accum._t.mul_(self._moving_rate).add_(cur)
                self._state._t.mul_(self._moving_rate).add_(1.0)
                self._scale._t.copy_(self._accum._t / self._state._t)
        return _w(fake_quant_dequant(x, self._scale._t.to(x.device).reshape(()), self._bit_length))

    def bit_length(self):
        return self._bit_length

    def quant_axis(self):
        return -1

    def scales(self):
        return self._scale

    def zero_points(self):
        return None


class FakeQuanterWithAbsMaxObserver(QuanterFactory):
    def __init__(self, moving_rate=0.9, bit_length=8, dtype="float32", name=None):
        super().__init__(name=name, moving_rate=moving_rate, bit_length=bit_length, dtype=dtype)

    def _get_class(self):
        return FakeQuanterWithAbsMaxObserverLayer


__all__ = ["FakeQuanterWithAbsMaxObserver"]
