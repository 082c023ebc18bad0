"""paddle.sparse.nn layers (reference: python/paddle/sparse/nn/layer/{activation,conv,norm,pooling}.py).
Layers hold dense parameters and run the functional sparse ops on COO / CSR inputs."""
from __future__ import annotations

import math

from ...framework.tensor import Tensor
from ...nn.layer.common import BatchNorm1D as _BN1D
from ...nn.layer.common import SyncBatchNorm as _SyncBN
from ...nn.layer.layers import Layer
from .. import ops as _ops
from ..creation import _u, to_coo_torch
from . import functional  # noqa: F401
from . import functional as F

_w = Tensor._wrap


class ReLU(Layer):
    def forward(self, x):
        return F.relu(x)


class ReLU6(Layer):
    def forward(self, x):
        return F.relu6(x)


class LeakyReLU(Layer):
    def __init__(self, negative_slope=0.01, name=None):
        super().__init__()
        self._slope = negative_slope

    def forward(self, x):
        return F.leaky_relu(x, self._slope)


class Softmax(Layer):
    def __init__(self, axis=-1, name=None):
        super().__init__()
        self._axis = axis

    def forward(self, x):
        return F.softmax(x, self._axis)


class _Conv(Layer):
    _ND, _SUBM = 3, False

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 padding_mode="zeros", key=None, weight_attr=None, bias_attr=None, data_format=None):
        super().__init__()
        nd = self._ND
        ks = tuple(kernel_size) if isinstance(kernel_size, (list, tuple)) else (kernel_size,) * nd
        self._stride, self._padding, self._dilation, self._groups = stride, padding, dilation, groups
        fan_in = in_channels * math.prod(ks)
        from ...nn import initializer as I

        bound = 1.0 / math.sqrt(fan_in)
        self.weight = self.create_parameter(list(ks) + [in_channels, out_channels], attr=weight_attr,
                                            default_initializer=I.Uniform(-bound, bound))
        self.bias = None if bias_attr is False else self.create_parameter(
            [out_channels], attr=bias_attr, is_bias=True, default_initializer=I.Uniform(-bound, bound))

    def forward(self, x):
        return F._conv(x, self.weight, self.bias, self._stride, self._padding, self._dilation, self._groups,
                       self._SUBM, self._ND, None)


class Conv3D(_Conv):
    _ND, _SUBM = 3, False


class SubmConv3D(_Conv):
    _ND, _SUBM = 3, True


class Conv2D(_Conv):
    _ND, _SUBM = 2, False


class SubmConv2D(_Conv):
    _ND, _SUBM = 2, True


class MaxPool3D(Layer):
    def __init__(self, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False, data_format="NDHWC",
                 name=None):
        super().__init__()
        self._args = (kernel_size, stride, padding)

    def forward(self, x):
        return F.max_pool3d(x, *self._args)


class BatchNorm(_BN1D):
    """BatchNorm over the channel values [nnz, C] of a COO tensor (statistics over the ACTIVE sites only, as the
    reference's sparse batch_norm)."""

    def __init__(self, num_features, momentum=0.9, epsilon=1e-5, weight_attr=None, bias_attr=None,
                 data_format="NDHWC", use_global_stats=None, name=None):
        super().__init__(num_features, momentum=momentum, epsilon=epsilon, weight_attr=weight_attr,
                         bias_attr=bias_attr)

    def forward(self, x):
        c = to_coo_torch(_u(x))
        out = super().forward(_w(c.values()))._t
        return _w(_ops._rebuild(c, out))


class SyncBatchNorm(_SyncBN):
    """Cross-rank BatchNorm over the active sites' channel values."""

    def __init__(self, num_features, momentum=0.9, epsilon=1e-5, weight_attr=None, bias_attr=None,
                 data_format="NCHW", name=None):
        super().__init__(num_features, momentum=momentum, epsilon=epsilon, weight_attr=weight_attr,
                         bias_attr=bias_attr, data_format="NC")

    def forward(self, x):
        c = to_coo_torch(_u(x))
        out = super().forward(_w(c.values()))._t
        return _w(_ops._rebuild(c, out))

    @classmethod
    def convert_sync_batchnorm(cls, layer):
        for name, sub in list(layer.named_children()) if hasattr(layer, "named_children") else []:
            setattr(layer, name, cls.convert_sync_batchnorm(sub))
        if isinstance(layer, BatchNorm):
            return cls(layer._num_features, layer._momentum, layer._epsilon)
        return layer
