"""Fake-quantization layers (reference: python/paddle/nn/quant/quant_layers.py — FakeQuantAbsMax :69,
FakeQuantMovingAverageAbsMax :172, FakeQuantChannelWiseAbsMax :310, MovingAverageAbsMaxScale :424,
QuantizedConv2D :544, QuantizedLinear :769, QuantizedMatmul :1060, MAOutputScaleLayer :1126).

Quantize-dequantize is ``round(clip(x / s, -1, 1) * qmax) * s / qmax`` with a straight-through
gradient (the reference's fake_quantize_dequantize_* grad kernels pass dout through unchanged).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ...framework.tensor import Tensor
from ..layer.layers import Layer

_w = Tensor._wrap


def _t(x):
    return x._t if isinstance(x, Tensor) else x


class _QDQ(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, scale, qmax):
        s = torch.clamp(scale.to(torch.float32), min=1e-12)
        xf = x.float()
        q = torch.round(torch.clamp(xf / s, -1.0, 1.0) * qmax)
        return (q * s / qmax).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g, None, None


def fake_quant_dequant(x, scale, bits=8, axis=None):
    """Straight-through fake quant-dequant of a torch tensor; ``scale`` is scalar or per-``axis``."""
    s = scale
    if axis is not None and s.dim() == 1 and s.numel() > 1:
        shp = [1] * x.dim()
        shp[axis] = -1
        s = s.reshape(shp)
    return _QDQ.apply(x, s, float(2 ** (bits - 1) - 1))


class FakeQuantAbsMax(Layer):
    """Per-tensor abs-max scale computed from the current batch."""

    def __init__(self, name=None, quant_bits=8, dtype="float32", quant_on_weight=False, reduce_type=None):
        super().__init__()
        self._quant_bits, self._reduce_type = quant_bits, reduce_type
        self.register_buffer("_scale", _w(torch.zeros(1)))

    def forward(self, input):
        x = _t(input)
        s = x.detach().abs().max().float().reshape(1)
        if self._reduce_type == "max":
            from ...distributed import collective as C

            if C.get_world_size() > 1:
                C._all_reduce_torch(s, op="max")
        self._scale._t.copy_(s)
        return _w(fake_quant_dequant(x, s.reshape(()), self._quant_bits))


class FakeQuantMovingAverageAbsMax(Layer):
    """scale = accum / state with accum = rate*accum + absmax(x), state = rate*state + 1 (training);
    the stored scale at eval."""

    def __init__(self, name=None, moving_rate=0.9, quant_bits=8, dtype="float32", reduce_type=None):
        super().__init__()
        self._moving_rate, self._quant_bits, self._reduce_type = moving_rate, quant_bits, reduce_type
        self.register_buffer("_scale", _w(torch.full((1,), 0.001)))
        self.register_buffer("_state", _w(torch.ones(1)))
        self._state._t.zero_()
        self.register_buffer("_accum", _w(torch.zeros(1)))

    def forward(self, input):
        x = _t(input)
        if self.training:
            with torch.no_grad():
                cur = x.detach().abs().max().float().reshape(1).to(self._accum._t.device)
                if self._reduce_type == "max":
                    from ...distributed import collective as C

                    if C.get_world_size() > 1:
                        C._all_reduce_torch(cur, op="max")
                self._accum._t.mul_(self._moving_rate).add_(cur)
                self._state._t.mul_(self._moving_rate).add_(1.0)
                self._scale._t.copy_(self._accum._t / self._state._t)
        return _w(fake_quant_dequant(x, self._scale._t.to(x.device).reshape(()), self._quant_bits))


class FakeQuantChannelWiseAbsMax(Layer):
    def __init__(self, name=None, channel_num=None, quant_bits=8, quant_axis=0, dtype="float32",
                 quant_on_weight=False, reduce_type=None):
        super().__init__()
        self._quant_bits, self._quant_axis = quant_bits, quant_axis
        self.register_buffer("_scale", _w(torch.zeros(channel_num or 1)))

    def forward(self, input):
        x = _t(input)
        dims = [d for d in range(x.dim()) if d != self._quant_axis]
        s = x.detach().abs().amax(dim=dims).float()
        if self._scale._t.shape != s.shape:
            self._scale._t = torch.zeros_like(s)
        self._scale._t.copy_(s)
        return _w(fake_quant_dequant(x, s, self._quant_bits, self._quant_axis))


class MovingAverageAbsMaxScale(Layer):
    """Observes the moving-average abs-max of its input (output unchanged)."""

    def __init__(self, name=None, moving_rate=0.9, dtype="float32", reduce_type=None):
        super().__init__()
        self._moving_rate = moving_rate
        self.register_buffer("_scale", _w(torch.zeros(1)))
        self.register_buffer("_state", _w(torch.zeros(1)))
        self.register_buffer("_accum", _w(torch.zeros(1)))

    def forward(self, input):
        if self.training:
            with torch.no_grad():
                cur = _t(input).detach().abs().max().float().reshape(1).to(self._accum._t.device)
                self._accum._t.mul_(self._moving_rate).add_(cur)
                self._state._t.mul_(self._moving_rate).add_(1.0)
                self._scale._t.copy_(self._accum._t / self._state._t)
        return input


MAOutputScaleLayer = None  # defined below (needs MovingAverageAbsMaxScale)


class MAOutputScaleLayer(Layer):  # noqa: F811
    def __init__(self, layer=None, moving_rate=0.9, name=None, dtype="float32", reduce_type=None):
        super().__init__()
        self._layer = layer
        self._ma_output_scale = MovingAverageAbsMaxScale(name, moving_rate, dtype, reduce_type)

    def forward(self, *inputs, **kwargs):
        out = self._layer(*inputs, **kwargs)
        if isinstance(out, (list, tuple)):
            return out
        return self._ma_output_scale(out)


class FakeQuantMAOutputScaleLayer(Layer):
    def __init__(self, layer, weight_bits=8, activation_bits=8, moving_rate=0.9, name=None, reduce_type=None,
                 *args, **kwargs):
        super().__init__()
        self._layer = layer
        self._fake_quant_output = FakeQuantMovingAverageAbsMax(name, moving_rate, activation_bits,
                                                               reduce_type=reduce_type)

    def forward(self, *inputs, **kwargs):
        out = self._layer(*inputs, **kwargs)
        if isinstance(out, (list, tuple)):
            return out
        return self._fake_quant_output(out)


def _get_fake_quant_type(quant_type, **kw):
    bits = kw.get("quant_bits", 8)
    if quant_type == "abs_max":
        return FakeQuantAbsMax(quant_bits=bits, reduce_type=kw.get("reduce_type"))
    if quant_type == "moving_average_abs_max":
        return FakeQuantMovingAverageAbsMax(moving_rate=kw.get("moving_rate", 0.9), quant_bits=bits,
                                            reduce_type=kw.get("reduce_type"))
    if quant_type == "channel_wise_abs_max":
        return FakeQuantChannelWiseAbsMax(channel_num=kw.get("channel_num"), quant_bits=bits,
                                          quant_axis=kw.get("quant_axis", 0), reduce_type=kw.get("reduce_type"))
    raise ValueError(f"unknown fake quant type {quant_type!r}")


class QuantizedLinear(Layer):
    """Linear with fake-quantized weight (per-channel along out features by default) and input."""

    def __init__(self, layer, weight_bits=8, activation_bits=8, moving_rate=0.9,
                 weight_quantize_type="abs_max", activation_quantize_type="abs_max", weight_pre_layer=None,
                 act_pre_layer=None, weight_quant_layer=None, act_quant_layer=None):
        super().__init__()
        self.weight, self.bias = layer.weight, layer.bias
        out_features = self.weight.shape[1]
        self._fake_quant_weight = weight_quant_layer() if weight_quant_layer else _get_fake_quant_type(
            weight_quantize_type, quant_bits=weight_bits, channel_num=out_features, quant_axis=1,
            moving_rate=moving_rate)
        self._fake_quant_input = act_quant_layer() if act_quant_layer else _get_fake_quant_type(
            activation_quantize_type, quant_bits=activation_bits, moving_rate=moving_rate)
        self._act_preprocess = act_pre_layer() if act_pre_layer else None
        self._weight_preprocess = weight_pre_layer() if weight_pre_layer else None

    def forward(self, input):
        if self._act_preprocess is not None:
            input = self._act_preprocess(input)
        qx = self._fake_quant_input(input)
        w = self.weight if self._weight_preprocess is None else self._weight_preprocess(self.weight)
        qw = self._fake_quant_weight(w)
        y = _t(qx) @ _t(qw)
        if self.bias is not None:
            y = y + _t(self.bias)
        return _w(y)


class QuantizedConv2D(Layer):
    def __init__(self, layer, weight_bits=8, activation_bits=8, moving_rate=0.9,
                 weight_quantize_type="abs_max", activation_quantize_type="abs_max", weight_pre_layer=None,
                 act_pre_layer=None, weight_quant_layer=None, act_quant_layer=None):
        super().__init__()
        self._layer = layer
        self.weight, self.bias = layer.weight, layer.bias
        self._fake_quant_weight = weight_quant_layer() if weight_quant_layer else _get_fake_quant_type(
            weight_quantize_type, quant_bits=weight_bits, channel_num=self.weight.shape[0], quant_axis=0,
            moving_rate=moving_rate)
        self._fake_quant_input = act_quant_layer() if act_quant_layer else _get_fake_quant_type(
            activation_quantize_type, quant_bits=activation_bits, moving_rate=moving_rate)

    def forward(self, input):
        from ..functional.conv import conv2d

        qx = self._fake_quant_input(input)
        qw = self._fake_quant_weight(self.weight)
        L = self._layer
        return conv2d(qx, qw, self.bias, L._stride, L._padding, L._dilation, L._groups, L._data_format)


class QuantizedMatmul(Layer):
    def __init__(self, layer=None, weight_bits=8, activation_bits=8, moving_rate=0.9,
                 activation_quantize_type="abs_max", act_pre_layer=None, act_quant_layer=None, **kw):
        super().__init__()
        mk = (lambda: act_quant_layer()) if act_quant_layer else (lambda: _get_fake_quant_type(  # noqa: E731
            activation_quantize_type, quant_bits=activation_bits, moving_rate=moving_rate))
        self._fake_quant_x, self._fake_quant_y = mk(), mk()

    def forward(self, x, y, transpose_x=False, transpose_y=False, name=None):
        a, b = _t(self._fake_quant_x(x)), _t(self._fake_quant_y(y))
        if transpose_x:
            a = a.transpose(-1, -2)
        if transpose_y:
            b = b.transpose(-1, -2)
        return _w(torch.matmul(a, b))
