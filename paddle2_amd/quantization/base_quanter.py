"""BaseQuanter (reference: python/paddle/quantization/base_quanter.py): the interface every quanter layer
implements — forward (fake-quantize or observe), scales, zero points, quant axis and bit length."""
from __future__ import annotations

import abc

from ..nn.layer.layers import Layer


class BaseQuanter(Layer, metaclass=abc.ABCMeta):
    def __init__(self):
        super().__init__()

    @abc.abstractmethod
    def forward(self, input):
        ...

    @abc.abstractmethod
    def scales(self):
        ...

    @abc.abstractmethod
    def zero_points(self):
        ...

    @abc.abstractmethod
    def quant_axis(self):
        ...

    @abc.abstractmethod
    def bit_length(self):
        ...
