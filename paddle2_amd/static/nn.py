"""paddle.static.nn: layer helpers that create parameters and record ops (reference: static/nn/common.py)."""
from __future__ import annotations

from .. import nn as _nn
from ..nn import functional as F


def fc(x, size, num_flatten_dims=1, weight_attr=None, bias_attr=None, activation=None, name=None):
    in_dim = 1
    for d in x.shape[num_flatten_dims:]:
        in_dim *= d
    lin = _nn.Linear(in_dim, size, weight_attr=weight_attr, bias_attr=bias_attr)
    h = x.reshape(list(x.shape[:num_flatten_dims]) + [in_dim]) if len(x.shape) > num_flatten_dims + 1 else x
    y = lin(h)
    if activation:
        y = getattr(F, activation)(y)
    return y


def embedding(input, size, is_sparse=False, is_distributed=False, padding_idx=None, param_attr=None, dtype="float32"):
    return _nn.Embedding(size[0], size[1], padding_idx=padding_idx, weight_attr=param_attr)(input)


def conv2d(input, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=1, param_attr=None,
           bias_attr=None, act=None, name=None, data_format="NCHW"):
    c = _nn.Conv2D(input.shape[1], num_filters, filter_size, stride, padding, dilation, groups,
                   weight_attr=param_attr, bias_attr=bias_attr, data_format=data_format)
    y = c(input)
    return getattr(F, act)(y) if act else y


def batch_norm(input, act=None, is_test=False, momentum=0.9, epsilon=1e-05, param_attr=None, bias_attr=None,
               data_layout="NCHW", name=None, **kw):
    bn = _nn.BatchNorm2D(input.shape[1], momentum=momentum, epsilon=epsilon, weight_attr=param_attr,
                         bias_attr=bias_attr, data_format=data_layout)
    if is_test:
        bn.eval()
    y = bn(input)
    return getattr(F, act)(y) if act else y


def layer_norm(input, scale=True, shift=True, begin_norm_axis=1, epsilon=1e-05, param_attr=None, bias_attr=None,
               act=None, name=None):
    shp = list(input.shape[begin_norm_axis:])
    ln = _nn.LayerNorm(shp, epsilon=epsilon, weight_attr=param_attr if scale else False,
                       bias_attr=bias_attr if shift else False)
    y = ln(input)
    return getattr(F, act)(y) if act else y
