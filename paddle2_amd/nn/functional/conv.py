"""Convolutions and pooling (reference: python/paddle/nn/functional/{conv,pooling}.py).

Conv/pool run on MIOpen through ATen ("Conv/BN start on MIOpen").
Paddle's ``padding`` may be an int, a list, or "SAME"/"VALID"; data_format NCHW or NHWC.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from ...framework.tensor import Tensor
from ...amp import amp_op as _amp_op  # noqa: E402

_wrap = Tensor._wrap


def _ntuple(v, n):
    if isinstance(v, (list, tuple)):
        v = [int(i) for i in v]
        if len(v) == 1:
            return v * n
        return v
    return [int(v)] * n


def _channel_last(fmt):
    return fmt in ("NHWC", "NLC", "NDHWC")


def _same_pad(t_spatial, k, s, d):
    pads = []
    for size, kk, ss, dd in zip(t_spatial, k, s, d):
        out = math.ceil(size / ss)
        total = max((out - 1) * ss + (kk - 1) * dd + 1 - size, 0)
        pads.append((total // 2, total - total // 2))
    return pads


def _resolve_padding(padding, n, spatial, k, s, d):
    """Returns (torch_padding_arg, explicit_pad_list_or_None)."""
    if isinstance(padding, str):
        p = padding.upper()
        if p == "VALID":
            return 0, None
        if p == "SAME":
            pads = _same_pad(spatial, k, s, d)
            if all(a == b for a, b in pads):
                return [a for a, _ in pads], None
            flat = []
            for a, b in reversed(pads):
                flat += [a, b]
            return 0, flat
    if isinstance(padding, (list, tuple)):
        p = [int(v) for v in (padding if not isinstance(padding[0], (list, tuple)) else
                              [x for pr in padding for x in pr])]
        if len(p) == n:
            return p, None
        if len(p) == 2 * n:
            if all(p[2 * i] == p[2 * i + 1] for i in range(n)):
                return [p[2 * i] for i in range(n)], None
            flat = []
            for i in reversed(range(n)):
                flat += [p[2 * i], p[2 * i + 1]]
            return 0, flat
        if len(p) == 2 * n + 4:  # includes batch/channel pairs
            p = p[4:]
            return [p[2 * i] for i in range(n)], None
        return p[:n], None
    return int(padding), None


def _conv(x, weight, bias, stride, padding, dilation, groups, data_format, n):
    t = x._t
    cl = _channel_last(data_format)
    if cl:
        t = t.movedim(-1, 1)
    k = list(weight._t.shape[2:])
    s = _ntuple(stride, n)
    d = _ntuple(dilation, n)
    tp, explicit = _resolve_padding(padding, n, list(t.shape[2:]), k, s, d)
    if explicit is not None:
        t = F.pad(t, explicit)
    fn = {1: F.conv1d, 2: F.conv2d, 3: F.conv3d}[n]
    out = fn(t, weight._t, None if bias is None else bias._t, s, tp, d, groups)
    if cl:
        out = out.movedim(1, -1)
    return _wrap(out)


@_amp_op("conv1d")
def conv1d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NCL", name=None):
    return _conv(x, weight, bias, stride, padding, dilation, groups, data_format, 1)


@_amp_op("conv2d")
def conv2d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NCHW", name=None):
    return _conv(x, weight, bias, stride, padding, dilation, groups, data_format, 2)


@_amp_op("conv3d")
def conv3d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NCDHW", name=None):
    return _conv(x, weight, bias, stride, padding, dilation, groups, data_format, 3)


def _conv_t(x, weight, bias, stride, padding, output_padding, dilation, groups, data_format, output_size, n):
    t = x._t
    cl = _channel_last(data_format)
    if cl:
        t = t.movedim(-1, 1)
    s = _ntuple(stride, n)
    d = _ntuple(dilation, n)
    k = list(weight._t.shape[2:])
    tp, _ = _resolve_padding(padding, n, list(t.shape[2:]), k, s, d)
    tp = _ntuple(tp, n)
    op = _ntuple(output_padding, n)
    if output_size is not None:
        osz = _ntuple(output_size, n)
        op = []
        for i in range(n):
            base = (t.shape[2 + i] - 1) * s[i] - 2 * tp[i] + d[i] * (k[i] - 1) + 1
            op.append(osz[i] - base)
    fn = {1: F.conv_transpose1d, 2: F.conv_transpose2d, 3: F.conv_transpose3d}[n]
    out = fn(t, weight._t, None if bias is None else bias._t, s, tp, op, groups, d)
    if cl:
        out = out.movedim(1, -1)
    return _wrap(out)


def conv1d_transpose(x, weight, bias=None, stride=1, padding=0, output_padding=0, groups=1, dilation=1,
                     output_size=None, data_format="NCL", name=None):
    return _conv_t(x, weight, bias, stride, padding, output_padding, dilation, groups, data_format, output_size, 1)


def conv2d_transpose(x, weight, bias=None, stride=1, padding=0, output_padding=0, dilation=1, groups=1,
                     output_size=None, data_format="NCHW", name=None):
    return _conv_t(x, weight, bias, stride, padding, output_padding, dilation, groups, data_format, output_size, 2)


def conv3d_transpose(x, weight, bias=None, stride=1, padding=0, output_padding=0, groups=1, dilation=1,
                     output_size=None, data_format="NCDHW", name=None):
    return _conv_t(x, weight, bias, stride, padding, output_padding, dilation, groups, data_format, output_size, 3)


# ------------------------------------------------------------------ pooling
def _pool(x, kernel_size, stride, padding, ceil_mode, data_format, n, kind, exclusive=True, return_mask=False,
          divisor_override=None):
    t = x._t
    cl = _channel_last(data_format)
    if cl:
        t = t.movedim(-1, 1)
    k = _ntuple(kernel_size, n)
    s = _ntuple(stride if stride is not None else kernel_size, n)
    tp, explicit = _resolve_padding(padding, n, list(t.shape[2:]), k, s, [1] * n)
    if explicit is not None:
        t = F.pad(t, explicit, value=float("-inf") if kind == "max" else 0.0)
    if kind == "max":
        fn = {1: F.max_pool1d, 2: F.max_pool2d, 3: F.max_pool3d}[n]
        r = fn(t, k, s, tp, 1, ceil_mode, return_mask)
        if return_mask:
            out, mask = r
            if cl:
                out, mask = out.movedim(1, -1), mask.movedim(1, -1)
            return _wrap(out), _wrap(mask)
        out = r
    else:
        fn = {1: F.avg_pool1d, 2: F.avg_pool2d, 3: F.avg_pool3d}[n]
        if n == 1:
            out = fn(t, k, s, tp, ceil_mode, not exclusive)
        else:
            out = fn(t, k, s, tp, ceil_mode, not exclusive, divisor_override)
    if cl:
        out = out.movedim(1, -1)
    return _wrap(out)


def max_pool1d(x, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False, name=None):
    return _pool(x, kernel_size, stride, padding, ceil_mode, "NCL", 1, "max", return_mask=return_mask)


def max_pool2d(x, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False, data_format="NCHW", name=None):
    return _pool(x, kernel_size, stride, padding, ceil_mode, data_format, 2, "max", return_mask=return_mask)


def max_pool3d(x, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False, data_format="NCDHW", name=None):
    return _pool(x, kernel_size, stride, padding, ceil_mode, data_format, 3, "max", return_mask=return_mask)


def avg_pool1d(x, kernel_size, stride=None, padding=0, exclusive=True, ceil_mode=False, name=None):
    return _pool(x, kernel_size, stride, padding, ceil_mode, "NCL", 1, "avg", exclusive)


def avg_pool2d(x, kernel_size, stride=None, padding=0, ceil_mode=False, exclusive=True, divisor_override=None,
               data_format="NCHW", name=None):
    return _pool(x, kernel_size, stride, padding, ceil_mode, data_format, 2, "avg", exclusive,
                 divisor_override=divisor_override)


def avg_pool3d(x, kernel_size, stride=None, padding=0, ceil_mode=False, exclusive=True, divisor_override=None,
               data_format="NCDHW", name=None):
    return _pool(x, kernel_size, stride, padding, ceil_mode, data_format, 3, "avg", exclusive,
                 divisor_override=divisor_override)


def _adaptive(x, output_size, data_format, n, kind, return_mask=False):
    t = x._t
    cl = _channel_last(data_format)
    if cl:
        t = t.movedim(-1, 1)
    if isinstance(output_size, (list, tuple)):
        output_size = [None if o is None else int(o) for o in output_size]
    if kind == "max":
        fn = {1: F.adaptive_max_pool1d, 2: F.adaptive_max_pool2d, 3: F.adaptive_max_pool3d}[n]
        r = fn(t, output_size, return_mask)
        if return_mask:
            o, m = r
            return _wrap(o.movedim(1, -1) if cl else o), _wrap(m.movedim(1, -1) if cl else m)
        out = r
    else:
        fn = {1: F.adaptive_avg_pool1d, 2: F.adaptive_avg_pool2d, 3: F.adaptive_avg_pool3d}[n]
        out = fn(t, output_size)
    if cl:
        out = out.movedim(1, -1)
    return _wrap(out)


def adaptive_avg_pool1d(x, output_size, name=None):
    return _adaptive(x, output_size, "NCL", 1, "avg")


def adaptive_avg_pool2d(x, output_size, data_format="NCHW", name=None):
    return _adaptive(x, output_size, data_format, 2, "avg")


def adaptive_avg_pool3d(x, output_size, data_format="NCDHW", name=None):
    return _adaptive(x, output_size, data_format, 3, "avg")


def adaptive_max_pool1d(x, output_size, return_mask=False, name=None):
    return _adaptive(x, output_size, "NCL", 1, "max", return_mask)


def adaptive_max_pool2d(x, output_size, return_mask=False, name=None):
    return _adaptive(x, output_size, "NCHW", 2, "max", return_mask)


def adaptive_max_pool3d(x, output_size, return_mask=False, name=None):
    return _adaptive(x, output_size, "NCDHW", 3, "max", return_mask)


def max_unpool2d(x, indices, kernel_size, stride=None, padding=0, data_format="NCHW", output_size=None, name=None):
    return _wrap(F.max_unpool2d(x._t, indices._t, kernel_size, stride, padding, output_size))


def lp_pool2d(x, norm_type, kernel_size, stride=None, ceil_mode=False, data_format="NCHW", name=None):
    return _wrap(F.lp_pool2d(x._t, norm_type, kernel_size, stride, ceil_mode))
