"""paddle.nn.initializer (reference: python/paddle/nn/initializer/*.py).

Initialisers act in place on a Parameter's torch storage; fan-in/fan-out follow Paddle's
convention for Linear weights stored ``[in_features, out_features]``.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ...framework.tensor import Tensor

_global_weight_init = None
_global_bias_init = None


def _fans(t: torch.Tensor):
    shape = t.shape
    if t.dim() == 0:
        return 1, 1
    if t.dim() == 1:
        return shape[0], shape[0]
    if t.dim() == 2:
        # Paddle Linear weights are [in, out]
        return shape[0], shape[1]
    receptive = int(np.prod(shape[2:]))
    return shape[1] * receptive, shape[0] * receptive


class Initializer:
    def __call__(self, param, block=None):
        t = param._t if isinstance(param, Tensor) else param
        with torch.no_grad():
            self._init(t)
        return param

    def _init(self, t):
        raise NotImplementedError


class Constant(Initializer):
    def __init__(self, value=0.0):
        self.value = value

    def _init(self, t):
        t.fill_(self.value)


class Normal(Initializer):
    def __init__(self, mean=0.0, std=1.0, name=None):
        self.mean, self.std = mean, std

    def _init(self, t):
        t.normal_(self.mean, self.std)


class TruncatedNormal(Initializer):
    def __init__(self, mean=0.0, std=1.0, a=-2.0, b=2.0, name=None):
        self.mean, self.std, self.a, self.b = mean, std, a, b

    def _init(self, t):
        torch.nn.init.trunc_normal_(t, self.mean, self.std, self.mean + self.a * self.std, self.mean + self.b * self.std)


class Uniform(Initializer):
    def __init__(self, low=-1.0, high=1.0, name=None):
        self.low, self.high = low, high

    def _init(self, t):
        t.uniform_(self.low, self.high)


class XavierNormal(Initializer):
    def __init__(self, fan_in=None, fan_out=None, gain=1.0, name=None):
        self.fan_in, self.fan_out, self.gain = fan_in, fan_out, gain

    def _init(self, t):
        fi, fo = _fans(t)
        fi = self.fan_in or fi
        fo = self.fan_out or fo
        std = self.gain * math.sqrt(2.0 / float(fi + fo))
        t.normal_(0.0, std)


class XavierUniform(Initializer):
    def __init__(self, fan_in=None, fan_out=None, gain=1.0, name=None):
        self.fan_in, self.fan_out, self.gain = fan_in, fan_out, gain

    def _init(self, t):
        fi, fo = _fans(t)
        fi = self.fan_in or fi
        fo = self.fan_out or fo
        limit = self.gain * math.sqrt(6.0 / float(fi + fo))
        t.uniform_(-limit, limit)


XavierInitializer = XavierUniform


def calculate_gain(nonlinearity, param=None):
    if nonlinearity in ("linear", "conv1d", "conv2d", "conv3d", "conv1d_transpose", "conv2d_transpose",
                        "conv3d_transpose", "sigmoid"):
        return 1.0
    if nonlinearity == "tanh":
        return 5.0 / 3
    if nonlinearity == "relu":
        return math.sqrt(2.0)
    if nonlinearity == "leaky_relu":
        slope = 0.01 if param is None else param
        return math.sqrt(2.0 / (1 + slope ** 2))
    if nonlinearity == "selu":
        return 3.0 / 4
    raise ValueError(nonlinearity)


class KaimingNormal(Initializer):
    def __init__(self, fan_in=None, negative_slope=0.0, nonlinearity="relu", mode="fan_in"):
        self.fan_in, self.slope, self.nl, self.mode = fan_in, negative_slope, nonlinearity, mode

    def _init(self, t):
        fi, fo = _fans(t)
        fan = self.fan_in or (fi if self.mode == "fan_in" else fo)
        gain = calculate_gain(self.nl, self.slope)
        t.normal_(0.0, gain / math.sqrt(float(fan)))


class KaimingUniform(Initializer):
    def __init__(self, fan_in=None, negative_slope=0.0, nonlinearity="relu", mode="fan_in"):
        self.fan_in, self.slope, self.nl, self.mode = fan_in, negative_slope, nonlinearity, mode

    def _init(self, t):
        fi, fo = _fans(t)
        fan = self.fan_in or (fi if self.mode == "fan_in" else fo)
        gain = calculate_gain(self.nl, self.slope)
        limit = gain * math.sqrt(3.0 / float(fan))
        t.uniform_(-limit, limit)


MSRAInitializer = KaimingNormal


class Assign(Initializer):
    def __init__(self, value, name=None):
        self.value = value

    def _init(self, t):
        v = self.value
        if isinstance(v, Tensor):
            v = v._t
        elif not isinstance(v, torch.Tensor):
            v = torch.as_tensor(np.asarray(v))
        t.copy_(v.reshape(t.shape).to(t.dtype))


NumpyArrayInitializer = Assign


class Orthogonal(Initializer):
    def __init__(self, gain=1.0, name=None):
        self.gain = gain

    def _init(self, t):
        torch.nn.init.orthogonal_(t, self.gain)


class Dirac(Initializer):
    def __init__(self, groups=1, name=None):
        self.groups = groups

    def _init(self, t):
        torch.nn.init.dirac_(t, self.groups)


class Bilinear(Initializer):
    def _init(self, t):
        shape = t.shape
        f = math.ceil(shape[3] / 2.0)
        c = (2 * f - 1 - f % 2) / (2.0 * f)
        w = torch.zeros(shape[2], shape[3])
        for i in range(shape[2]):
            for j in range(shape[3]):
                w[i, j] = (1 - abs(i / f - c)) * (1 - abs(j / f - c))
        t.copy_(w.expand(shape).to(t.dtype))


def set_global_initializer(weight_init, bias_init=None):
    global _global_weight_init, _global_bias_init
    _global_weight_init = weight_init
    _global_bias_init = bias_init


# lower-case aliases used by some Paddle code
constant = Constant
normal = Normal
uniform = Uniform
