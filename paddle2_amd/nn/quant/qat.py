"""QAT layers (reference: python/paddle/nn/quant/qat/linear.py QuantedLinear, conv.py QuantedConv2D):
the float layer's parameters, a weight quanter and an activation quanter from the QuantConfig."""
from __future__ import annotations

from ...framework.tensor import Tensor
from . import ConvertibleQuantedLayer


class QuantedLinear(ConvertibleQuantedLayer):
    def __init__(self, layer, q_config):
        super().__init__()
        self.weight, self.bias = layer.weight, layer.bias
        self.name = getattr(layer, "_name", None)
        self.weight_quanter = q_config.weight._instance(layer) if q_config.weight is not None else None
        self.activation_quanter = q_config.activation._instance(layer) if q_config.activation is not None else None

    def forward(self, input):
        from ..functional import linear

        x = self.activation_quanter(input) if self.activation_quanter is not None else input
        w = self.weight_quanter(self.weight) if self.weight_quanter is not None else self.weight
        return linear(x, w, self.bias)

    def weights_to_quanters(self):
        return [("weight", "weight_quanter")]

    def activation_quanters(self):
        return ["activation_quanter"]


class QuantedConv2D(ConvertibleQuantedLayer):
    def __init__(self, layer, q_config):
        super().__init__()
        self._layer = layer
        self.weight, self.bias = layer.weight, layer.bias
        self.weight_quanter = q_config.weight._instance(layer) if q_config.weight is not None else None
        self.activation_quanter = q_config.activation._instance(layer) if q_config.activation is not None else None

    def forward(self, input):
        from ..functional.conv import conv2d

        x = self.activation_quanter(input) if self.activation_quanter is not None else input
        w = self.weight_quanter(self.weight) if self.weight_quanter is not None else self.weight
        L = self._layer
        return conv2d(x, w, self.bias, L._stride, L._padding, L._dilation, L._groups, L._data_format)

    def weights_to_quanters(self):
        return [("weight", "weight_quanter")]

    def activation_quanters(self):
        return ["activation_quanter"]


__all__ = ["QuantedLinear", "QuantedConv2D", "Tensor"]
