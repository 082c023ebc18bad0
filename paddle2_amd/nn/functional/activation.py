"""Activations (reference: python/paddle/nn/functional/activation.py)."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ...framework.tensor import Tensor
from ...amp import amp_op as _amp_op  # noqa: E402

_wrap = Tensor._wrap


def relu(x, name=None):
    return _wrap(F.relu(x._t))


def relu_(x, name=None):
    F.relu_(x._t)
    return x


def relu6(x, name=None):
    return _wrap(F.relu6(x._t))


def leaky_relu(x, negative_slope=0.01, name=None):
    return _wrap(F.leaky_relu(x._t, negative_slope))


def leaky_relu_(x, negative_slope=0.01, name=None):
    F.leaky_relu_(x._t, negative_slope)
    return x


def prelu(x, weight, data_format="NCHW", name=None):
    t = x._t
    w = weight._t
    if data_format[-1] == "C" and t.dim() > 2 and w.numel() > 1:
        t = t.movedim(-1, 1)
        return _wrap(F.prelu(t, w).movedim(1, -1))
    return _wrap(F.prelu(t, w))


def rrelu(x, lower=1.0 / 8.0, upper=1.0 / 3.0, training=True, name=None):
    return _wrap(F.rrelu(x._t, lower, upper, training))


def elu(x, alpha=1.0, name=None):
    return _wrap(F.elu(x._t, alpha))


def elu_(x, alpha=1.0, name=None):
    F.elu_(x._t, alpha)
    return x


def celu(x, alpha=1.0, name=None):
    return _wrap(F.celu(x._t, alpha))


def selu(x, scale=1.0507009873554804934193349852946, alpha=1.6732632423543772848170429916717, name=None):
    return _wrap(scale * torch.where(x._t > 0, x._t, alpha * (torch.exp(x._t) - 1)))


def gelu(x, approximate=False, name=None):
    """GPU bf16 / fp16: the native bias-activation kernel (csrc/kernels/fused_act.hip, erf or tanh form, its own
    backward) instead of ATen's GeluCUDAKernel / GeluBackward (reference phi/kernels/gpu/gelu_kernel.cu)."""
    t = x._t
    if t.is_cuda and t.dtype in (torch.bfloat16, torch.float16) and t.dim() >= 1 and t.shape[-1] % 8 == 0:
        from ...ops import _native as N
        from ...ops import torch_ops as T

        if not isinstance(t, T._DTensor) and N.use_native(t):
            from ...ops import fused as FU

            return _wrap(FU.bias_act(t, None, "gelu_tanh" if approximate else "gelu"))
    return _wrap(F.gelu(t, approximate="tanh" if approximate else "none"))


def silu(x, name=None):
    return _wrap(F.silu(x._t))


swish = silu


def mish(x, name=None):
    return _wrap(F.mish(x._t))


def sigmoid(x, name=None):
    return _wrap(torch.sigmoid(x._t))


def hardsigmoid(x, slope=0.1666667, offset=0.5, name=None):
    return _wrap(torch.clamp(x._t * slope + offset, 0.0, 1.0))


def hardswish(x, name=None):
    return _wrap(F.hardswish(x._t))


def hardtanh(x, min=-1.0, max=1.0, name=None):
    return _wrap(F.hardtanh(x._t, min, max))


def hardshrink(x, threshold=0.5, name=None):
    return _wrap(F.hardshrink(x._t, threshold))


def softshrink(x, threshold=0.5, name=None):
    return _wrap(F.softshrink(x._t, threshold))


def tanhshrink(x, name=None):
    return _wrap(F.tanhshrink(x._t))


def thresholded_relu(x, threshold=1.0, value=0.0, name=None):
    return _wrap(torch.where(x._t > threshold, x._t, torch.full_like(x._t, value)))


def softplus(x, beta=1, threshold=20, name=None):
    return _wrap(F.softplus(x._t, beta, threshold))


def softsign(x, name=None):
    return _wrap(F.softsign(x._t))


def tanh(x, name=None):
    return _wrap(torch.tanh(x._t))


def tanh_(x, name=None):
    x._t.tanh_()
    return x


def log_sigmoid(x, name=None):
    return _wrap(F.logsigmoid(x._t))


def maxout(x, groups, axis=1, name=None):
    t = x._t
    shp = list(t.shape)
    ax = axis % t.dim()
    c = shp[ax]
    new = shp[:ax] + [c // groups, groups] + shp[ax + 1:]
    return _wrap(t.reshape(new).amax(ax + 1))


@_amp_op("softmax")
def softmax(x, axis=-1, dtype=None, name=None):
    t = x._t
    if dtype is not None:
        from ...framework.dtype import convert_dtype

        t = t.to(convert_dtype(dtype))
    return _wrap(torch.softmax(t, axis))


def softmax_(x, axis=-1, dtype=None, name=None):
    r = softmax(x, axis, dtype)
    x._t = r._t
    return x


@_amp_op("log_softmax")
def log_softmax(x, axis=-1, dtype=None, name=None):
    t = x._t
    if dtype is not None:
        from ...framework.dtype import convert_dtype

        t = t.to(convert_dtype(dtype))
    return _wrap(torch.log_softmax(t, axis))


def gumbel_softmax(x, temperature=1.0, hard=False, axis=-1, name=None):
    return _wrap(F.gumbel_softmax(x._t, tau=temperature, hard=hard, dim=axis))


def glu(x, axis=-1, name=None):
    return _wrap(F.glu(x._t, axis))


def swiglu(x, y=None, name=None):
    from ...ops import swiglu as _sw

    return _sw(x, y)
