"""paddle.nn.quant (reference: python/paddle/nn/quant/ — quantized_linear.py:56 weight_quantize,
:123 weight_dequantize, :183 weight_only_linear, :276 llm_int8_linear, :342 apply_per_channel_scale;
quant_layers.py fake-quant layers; format.py LinearQuanter/LinearDequanter/ConvertibleQuantedLayer;
stub.py Stub/QuanterStub; qat/ QuantedLinear/QuantedConv2D; functional_layers.py).

Weight-only formats (MI355X-native, no CUTLASS interleaving): for a [K, N] (in, out) weight
``weight_quantize`` returns int8 ``[N, K]`` (each output channel's K weights contiguous — the
layout the decode GEMV streams) or, for int4, ``[N/2, K]`` with channel 2i in the low and 2i+1 in
the high nibble; scales are per channel ``[N]`` or per group ``[K/group, N]``.
``weight_only_linear`` runs the HIP weight-only kernel for small token counts on the GPU
(csrc/kernels/weight_only.hip) and dequantize + GEMM otherwise.
"""
from __future__ import annotations

import abc

import torch

from ...framework.tensor import Tensor
from ..layer.layers import Layer
from .functional_layers import (FloatFunctionalLayer, add, concat, divide, flatten, matmul, multiply,  # noqa: F401
                                reshape, subtract, transpose)
from .quant_layers import (FakeQuantAbsMax, FakeQuantChannelWiseAbsMax, FakeQuantMAOutputScaleLayer,  # noqa: F401
                           FakeQuantMovingAverageAbsMax, MAOutputScaleLayer, MovingAverageAbsMaxScale,
                           QuantizedConv2D, QuantizedLinear, QuantizedMatmul, fake_quant_dequant)

_w = Tensor._wrap


def _t(x):
    return x._t if isinstance(x, Tensor) else x


# ----------------------------------------------------------------------------- weight-only quantization
def _absmax_scale(w, bits, group_size):
    qmax = float(2 ** (bits - 1) - 1)
    K, Nn = w.shape
    if group_size == -1:
        s = w.abs().amax(0) / qmax                             # [N]
        sx = s[None, :]
    else:
        g = w.reshape(-1, group_size, Nn).abs().amax(1) / qmax  # [K/g, N]
        s, sx = g, g.repeat_interleave(group_size, 0)[:K]
    s = torch.where(s == 0, torch.ones_like(s), s)
    sx = torch.where(sx == 0, torch.ones_like(sx), sx)
    return s, sx, qmax


def weight_quantize(x, algo="weight_only_int8", arch=None, group_size=-1):
    """x: [K, N] float -> (int8 weight [N, K] (int4: [N/2, K] packed), scale [N] or [K/group, N])."""
    if algo not in ("weight_only_int8", "weight_only_int4", "llm.int8"):
        raise ValueError(f"algo must be weight_only_int8 / weight_only_int4 / llm.int8, got {algo!r}")
    if group_size not in (-1, 64, 128):
        raise ValueError("group_size must be -1, 64 or 128")
    w = _t(x).float()
    if w.dim() != 2:
        raise ValueError("weight_quantize expects a 2-D [in, out] weight")
    bits = 4 if algo == "weight_only_int4" else 8
    s, sx, qmax = _absmax_scale(w, bits, group_size)
    q = torch.clamp(torch.round(w / sx), -qmax, qmax).to(torch.int8)   # [K, N]
    qt = q.t().contiguous()                                                # [N, K]
    if bits == 4:
        if qt.shape[0] % 2:
            raise ValueError("int4 weight-only quantization needs an even number of output channels")
        lo = qt[0::2].to(torch.int16) & 0xF
        hi = (qt[1::2].to(torch.int16) & 0xF) << 4
        qt = (lo | hi).to(torch.uint8).view(torch.int8)                  # [N/2, K]
    return _w(qt), _w(s.to(_t(x).dtype))


def _dequant(weight, scale, weight_dtype="int8", group_size=-1, out_dtype=torch.float32):
    from ...ops.weight_only import dequantize

    return dequantize(_t(weight), _t(scale), weight_dtype, group_size, out_dtype)  # [N, K]


def weight_dequantize(x, scale, algo="weight_only_int8", out_dtype="float16", group_size=-1):
    """Inverse of weight_quantize -> float [K, N]."""
    from ...framework.dtype import convert_dtype

    wd = "int4" if algo == "weight_only_int4" else "int8"
    return _w(_dequant(x, scale, wd, group_size, convert_dtype(out_dtype)).t().contiguous())


def weight_only_linear(x, weight, bias=None, weight_scale=None, weight_dtype="int8", arch=None, group_size=-1):
    """y = x @ dequant(weight)^T + bias; x [..., K], weight [N, K] int8 (or [N/2, K] int4)."""
    if weight_dtype not in ("int8", "int4"):
        raise ValueError("weight_dtype must be 'int8' or 'int4'")
    xt = _t(x)
    K = xt.shape[-1]
    from ...ops import weight_only as _wo

    y = _wo.weight_only_matmul(xt.reshape(-1, K), _t(weight), _t(weight_scale), weight_dtype, group_size,
                               None if bias is None else _t(bias))
    return _w(y.reshape(*xt.shape[:-1], y.shape[-1]))


def llm_int8_linear(x, weight, bias=None, weight_scale=None, threshold=6.0):
    """LLM.int8(): outlier input features (|x| > threshold in any row) run in floating point, the
    rest as int8 x int8 with per-row activation scales."""
    xt = _t(x)
    K = xt.shape[-1]
    x2 = xt.reshape(-1, K).float()
    wq = _t(weight).float()                            # [N, K]
    s = _t(weight_scale).float()
    outl = (x2.abs() > threshold).any(0)
    xin = torch.where(outl[None, :], torch.zeros_like(x2), x2)  # regular features only
    xs = xin.abs().amax(1, keepdim=True).clamp(min=1e-8) / 127.0
    xi = torch.round(xin / xs).clamp(-127, 127)
    y = (xi @ wq.t()) * xs * s[None, :]
    if outl.any():
        y = y + x2[:, outl] @ (wq[:, outl] * s[:, None]).t()
    y = y.to(xt.dtype).reshape(*xt.shape[:-1], -1)
    if bias is not None:
        y = y + _t(bias).to(y.dtype)
    return _w(y)


def apply_per_channel_scale(x, scales):
    return _w(_t(x) * _t(scales).to(_t(x).dtype))


# ----------------------------------------------------------------------------- fp8 fake quant
_FP8 = {"e4m3": (torch.float8_e4m3fn, 448.0), "e5m2": (torch.float8_e5m2, 57344.0)}


def fake_fp8_quant(input, scale, axis=-1, type="e4m3"):
    dt, mx = _FP8[type]
    x = _t(input)
    s = _t(scale).float()
    if s.dim() == 1 and axis != -1 and s.numel() > 1:
        shp = [1] * x.dim()
        shp[axis] = -1
        s = s.reshape(shp)
    return _w((x.float() / s * mx).clamp(-mx, mx).to(dt))


def fake_fp8_dequant(input, scale, axis=-1, type="e4m3"):
    _, mx = _FP8[type]
    x = _t(input)
    s = _t(scale).float()
    if s.dim() == 1 and axis != -1 and s.numel() > 1:
        shp = [1] * x.dim()
        shp[axis] = -1
        s = s.reshape(shp)
    return _w(x.float() * s / mx)


# ----------------------------------------------------------------------------- deploy format
class LinearQuanter(Layer):
    """Quantize to the integer grid (kept in float): round(x / scale * qmax) [+ zero point]."""

    def __init__(self, scales, zero_point=None, quant_axis=None, bit_length=8, group_size=128):
        super().__init__()
        self.register_buffer("_scales", _w(torch.as_tensor(_t(scales), dtype=torch.float32).clone()))
        zp = torch.zeros_like(self._scales._t) if zero_point is None else torch.as_tensor(_t(zero_point),
                                                                                         dtype=torch.float32)
        self.register_buffer("_zero_point", _w(zp))
        self._quant_axis = -1 if quant_axis is None else quant_axis
        self._bit_length, self._group_size = bit_length, group_size
        self._qmax = float(2 ** (bit_length - 1) - 1) if isinstance(bit_length, int) else \
            {(4, 3): 448.0, (5, 2): 57344.0}[tuple(bit_length)]

    def _bcast(self, t, x):
        if t.dim() == 0 or t.numel() == 1 or self._quant_axis == -1:
            return t.reshape(()) if t.numel() == 1 else t
        shp = [1] * x.dim()
        shp[self._quant_axis] = -1
        return t.reshape(shp)

    def forward(self, input):
        x = _t(input)
        s = self._bcast(self._scales._t, x)
        zp = self._bcast(self._zero_point._t, x)
        return _w(torch.clamp(torch.round(x.float() / s * self._qmax) + zp, -self._qmax - 1, self._qmax))

    @staticmethod
    def from_quanter(quanter):
        return LinearQuanter(quanter.scales(), quanter.zero_points(), quanter.quant_axis(), quanter.bit_length())


class LinearDequanter(LinearQuanter):
    def forward(self, input):
        x = _t(input).float()
        s = self._bcast(self._scales._t, x)
        zp = self._bcast(self._zero_point._t, x)
        return _w((x - zp) * s / self._qmax)

    @staticmethod
    def from_quanter(quanter):
        return LinearDequanter(quanter.scales(), quanter.zero_points(), quanter.quant_axis(), quanter.bit_length())


class LinearQuanterDequanter(Layer):
    def __init__(self, quanter, dequanter):
        super().__init__()
        self._quanter, self._dequanter = quanter, dequanter

    def forward(self, input):
        out = input
        if self._quanter is not None:
            out = self._quanter(out)
        if self._dequanter is not None:
            out = self._dequanter(out)
        return out

    @staticmethod
    def from_quanter(quanter):
        return LinearQuanterDequanter(LinearQuanter.from_quanter(quanter), LinearDequanter.from_quanter(quanter))


class ConvertibleQuantedLayer(Layer, metaclass=abc.ABCMeta):
    """A QAT layer that can be converted for deployment: weights are replaced by their quantized
    integer values (dequantized at run time) and activation quanters become quant/dequant pairs."""

    def __init__(self):
        super().__init__()
        self.converted = False

    @abc.abstractmethod
    def weights_to_quanters(self):
        ...

    @abc.abstractmethod
    def activation_quanters(self):
        ...

    def _convert_quanter_to_qdq(self, name):
        q = getattr(self, name)
        if q is None:
            return None
        qdq = LinearQuanterDequanter.from_quanter(q)
        setattr(self, name, qdq)
        self._sub_layers[name] = qdq
        return qdq

    def _quant_weights(self, linear_quanter, weight):
        with torch.no_grad():
            q = linear_quanter(weight)
            weight._t.copy_(q._t.to(weight._t.dtype))

    def _convert(self, remain_weight=False):
        for wname, qname in self.weights_to_quanters():
            qdq = self._convert_quanter_to_qdq(qname)
            if not remain_weight and qdq is not None:
                self._quant_weights(qdq._quanter, getattr(self, wname))
                qdq._quanter = None
        for qname in self.activation_quanters():
            self._convert_quanter_to_qdq(qname)
        self.converted = True


class Stub(Layer):
    """Marks a point in forward() where an activation quanter/observer should be inserted."""

    def __init__(self, observer=None):
        super().__init__()
        self._observer = observer

    def forward(self, input):
        return input


class QuanterStub(Layer):
    def __init__(self, layer, q_config):
        super().__init__()
        self._observer = None
        if q_config.activation is not None:
            self._observer = q_config.activation._instance(layer)

    def forward(self, input):
        return self._observer(input) if self._observer is not None else input


from .qat import QuantedConv2D, QuantedLinear  # noqa: E402,F401

__all__ = ["weight_quantize", "weight_dequantize", "weight_only_linear", "llm_int8_linear", "apply_per_channel_scale",
           "fake_fp8_quant", "fake_fp8_dequant", "Stub", "QuanterStub", "LinearQuanter", "LinearDequanter",
           "LinearQuanterDequanter", "ConvertibleQuantedLayer", "QuantedLinear", "QuantedConv2D",
           "FakeQuantAbsMax", "FakeQuantMovingAverageAbsMax", "FakeQuantChannelWiseAbsMax",
           "MovingAverageAbsMaxScale", "QuantizedLinear", "QuantizedConv2D", "QuantizedMatmul"]
