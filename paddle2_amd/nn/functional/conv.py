"""Convolutions and pooling (reference: python/paddle/nn/functional/{conv,pooling}.py).

Conv/pool run on MIOpen through ATen ("Conv/BN start on MIOpen"), except channels-last 1x1
convolutions (two of the three convs of every ResNet bottleneck), which are GEMMs on the native MFMA kernels.
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


from ...ops import conv_gemm as _CG  # noqa: E402


def _conv1x1_native(t_nhwc, weight, bias, stride, groups, dilation):
    """The native 1x1 path applies: GPU bf16, NHWC, a 1x1 kernel without padding or groups, channel counts the
    GEMM's 16-B chunks take (multiples of 8)."""
    from ...ops import _native as N

    w = weight._t
    return (_CG.MODE in ("native", "auto") and t_nhwc.is_cuda and t_nhwc.dtype == torch.bfloat16
            and w.dtype == t_nhwc.dtype and groups == 1 and tuple(w.shape[2:]) == (1, 1)
            and all(dd == 1 for dd in dilation) and w.shape[1] % 8 == 0 and w.shape[0] % 8 == 0
            and (bias is None or bias._t.dtype == t_nhwc.dtype) and N.use_native(t_nhwc)
            and _CG.route("1x1", t_nhwc, w, stride, [0, 0]))


def _conv(x, weight, bias, stride, padding, dilation, groups, data_format, n):
    t = x._t
    cl = _channel_last(data_format)
    if cl and n == 2 and padding in (0, [0, 0], (0, 0), "VALID", "valid"):
        s2, d2 = _ntuple(stride, 2), _ntuple(dilation, 2)
        if _conv1x1_native(t, weight, bias, s2, groups, d2):
            if s2 != [1, 1]:
                t = t[:, ::s2[0], ::s2[1], :]
            if not t.is_contiguous():
                t = t.contiguous()
            return _wrap(_CG.Conv1x1Fn.apply(t, weight._t, None if bias is None else bias._t))
    if cl and n == 2:
        s2, d2 = _ntuple(stride, 2), _ntuple(dilation, 2)
        pad = padding if isinstance(padding, str) else _ntuple(padding, 2)
        if isinstance(pad, str):
            pad = [1, 1] if pad.upper() == "SAME" and s2 == [1, 1] else None
        if pad is not None and _CG.eligible_3x3(t, weight._t, s2, pad, d2, groups):
            y = _CG.Conv3x3Fn.apply(t.contiguous(), weight._t)
            if bias is not None:
                y = y + bias._t
            return _wrap(y)
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


def lp_pool1d(x, norm_type, kernel_size, stride=None, padding=0, ceil_mode=False, data_format="NCL", name=None):
    """Power-average pooling (reference nn/functional/pooling.py lp_pool1d): (sum x^p)^(1/p) per window."""
    t = x._t
    if padding:
        t = F.pad(t, (padding, padding))
    return _wrap(F.lp_pool1d(t, float(norm_type), kernel_size, stride, ceil_mode))


def max_unpool1d(x, indices, kernel_size, stride=None, padding=0, data_format="NCL", output_size=None, name=None):
    return _wrap(F.max_unpool1d(x._t, indices._t, kernel_size, stride, padding, output_size))


def max_unpool3d(x, indices, kernel_size, stride=None, padding=0, data_format="NCDHW", output_size=None, name=None):
    return _wrap(F.max_unpool3d(x._t, indices._t, kernel_size, stride, padding, output_size))


def _fractional_bounds(inp, out, pool, u):
    """Window [start, end) per output index, the reference's pseudo-random sequence
    (phi/kernels/funcs/pooling.h:142 FractionalRationalU / StartIndex / EndIndex)."""
    alpha = float(inp - pool) / (out - (1 if pool > 0 else 0))
    if pool <= 0:
        base = inp // out
        u = u * min((base + 2) / alpha - 1, (inp + 1 - base) / alpha - (out - 1))
    st, en = [], []
    for i in range(out):
        s0 = int((i + u) * alpha) - int(u * alpha)
        e0 = s0 + pool if pool > 0 else int((i + 1 + u) * alpha) - int(u * alpha)
        st.append(max(s0, 0))
        en.append(min(e0, inp))
    return st, en


def _fractional(x, output_size, kernel_size, random_u, return_mask, n):
    t = x._t
    sp = list(t.shape[2:])
    outs = [output_size] * n if isinstance(output_size, int) else list(output_size)
    pools = [0] * n if kernel_size is None else ([kernel_size] * n if isinstance(kernel_size, int) else list(kernel_size))
    if random_u is None or float(random_u) == 0.0:
        u = float(torch.rand(()))
    else:
        u = float(random_u)
        if not 0.0 < u < 1.0:
            raise ValueError("random_u must be in (0, 1)")
    # per dim: gather index [out, win] (clamped) + validity mask, then a masked max over all window dims
    y, flat = t, None
    idx_dims, masks = [], []
    for d in range(n):
        st, en = _fractional_bounds(sp[d], outs[d], pools[d], u)
        win = max(e - s for s, e in zip(st, en))
        ar = torch.arange(win, device=t.device)
        s_t = torch.tensor(st, device=t.device)[:, None]
        e_t = torch.tensor(en, device=t.device)[:, None]
        idx = (s_t + ar).clamp_max(sp[d] - 1)
        idx_dims.append(idx)
        masks.append((s_t + ar) < e_t)
    # y[N, C, o0, w0, o1, w1, ...]
    for d in range(n):
        ax = 2 + 2 * d
        y = y.index_select(ax, idx_dims[d].reshape(-1)).unflatten(ax, idx_dims[d].shape)
    valid = masks[0]
    lin = idx_dims[0]
    for d in range(1, n):
        valid = valid[(...,) + (None, None)] & masks[d][(None, None) * d]
        lin = lin[(...,) + (None, None)] * sp[d] + idx_dims[d][(None, None) * d]
    # move window axes last: [N, C, o0, o1, ..., w0, w1, ...]
    perm = [0, 1] + [2 + 2 * d for d in range(n)] + [3 + 2 * d for d in range(n)]
    y = y.permute(perm).flatten(2 + n)
    pv = list(range(0, 2 * n, 2)) + list(range(1, 2 * n, 2))
    valid = valid.permute(pv).flatten(n)
    lin = lin.permute(pv).flatten(n)
    y = y.masked_fill(~valid, float("-inf"))
    val, arg = y.max(-1)
    if not return_mask:
        return _wrap(val)
    mask = torch.gather(lin.expand(*val.shape, lin.shape[-1]), -1, arg.unsqueeze(-1)).squeeze(-1)
    return _wrap(val), _wrap(mask)


def fractional_max_pool2d(x, output_size, kernel_size=None, random_u=None, return_mask=False, name=None):
    """Fractional max pooling (Graham 2014; reference nn/functional/pooling.py): pseudo-random window
    boundaries, one shared ``random_u`` in (0, 1) makes the pooling sequence reproducible."""
    return _fractional(x, output_size, kernel_size, random_u, return_mask, 2)


def fractional_max_pool3d(x, output_size, kernel_size=None, random_u=None, return_mask=False, name=None):
    return _fractional(x, output_size, kernel_size, random_u, return_mask, 3)
