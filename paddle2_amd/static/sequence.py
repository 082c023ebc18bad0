"""LoD sequences and the static.nn sequence ops (reference python/paddle/static/nn/sequence_lod.py; kernels
phi/kernels/*/sequence_pool_kernel, sequence_softmax, sequence_expand, sequence_conv).

A LoD tensor here is an ordinary tensor whose rows are the concatenated sequences plus a level-of-detail offset
list set with ``Tensor.set_lod([[0, 3, 5, ...]])`` (or ``set_recursive_sequence_lengths([[3, 2, ...]])``) — the
reference's LoDTensor layout.  The ops read the last LoD level.
"""
from __future__ import annotations

import torch

from ..framework.tensor import Tensor


def _raw(x):
    return x._t if isinstance(x, Tensor) else x


def _offsets(x):
    lod = getattr(x, "_lod", None)
    if not lod:
        raise ValueError("sequence op: the input has no LoD (set it with Tensor.set_lod)")
    return [int(v) for v in lod[-1]]


def _with_lod(t, lod):
    out = Tensor._wrap(t)
    out._lod = lod
    return out


def sequence_pool(input, pool_type, is_test=False, pad_value=0.0):  # noqa: A002
    """Pool every sequence's rows: sum / average / sqrt (sum / sqrt(len)) / max / min / first / last; empty
    sequences give pad_value.  [T, D] -> [N, D]."""
    r = _raw(input)
    off = _offsets(input)
    rows = []
    pt = pool_type.lower()
    for a, b in zip(off[:-1], off[1:]):
        seg = r[a:b]
        if b == a:
            rows.append(torch.full(r.shape[1:], pad_value, dtype=r.dtype, device=r.device))
        elif pt == "sum":
            rows.append(seg.sum(0))
        elif pt == "average":
            rows.append(seg.mean(0))
        elif pt == "sqrt":
            rows.append(seg.sum(0) / (b - a) ** 0.5)
        elif pt == "max":
            rows.append(seg.max(0).values)
        elif pt == "min":
            rows.append(seg.min(0).values)
        elif pt == "first":
            rows.append(seg[0])
        elif pt == "last":
            rows.append(seg[-1])
        else:
            raise ValueError(f"sequence_pool: unknown pool_type {pool_type!r}")
    return Tensor._wrap(torch.stack(rows))


def sequence_first_step(input):  # noqa: A002
    return sequence_pool(input, "first")


def sequence_last_step(input):  # noqa: A002
    return sequence_pool(input, "last")


def sequence_softmax(input, use_cudnn=False, name=None):  # noqa: A002
    """Softmax over each sequence's rows of a [T, 1] (or [T]) input."""
    r = _raw(input)
    off = _offsets(input)
    flat = r.reshape(-1)
    out = torch.empty_like(flat)
    for a, b in zip(off[:-1], off[1:]):
        if b > a:
            out[a:b] = torch.softmax(flat[a:b].float(), 0).to(flat.dtype)
    return _with_lod(out.reshape(r.shape), input._lod)


def sequence_expand(x, y, ref_level=-1, name=None):
    """Repeat x's i-th sequence (or row, without LoD) len_i times where len_i are y's sequence lengths at
    ref_level; the result carries the expanded LoD."""
    xr = _raw(x)
    yoff = [int(v) for v in y._lod[ref_level]]
    reps = [b - a for a, b in zip(yoff[:-1], yoff[1:])]
    xlod = getattr(x, "_lod", None)
    xoff = [int(v) for v in xlod[-1]] if xlod else list(range(xr.shape[0] + 1))
    pieces, new = [], [0]
    for i, n in enumerate(reps):
        seg = xr[xoff[i]:xoff[i + 1]]
        for _ in range(n):
            pieces.append(seg)
            new.append(new[-1] + seg.shape[0])
    out = torch.cat(pieces, 0) if pieces else xr[:0]
    return _with_lod(out, [new])


def sequence_conv(input, num_filters, filter_size=3, filter_stride=1, padding=True, padding_start=None,  # noqa: A002
                  bias_attr=None, param_attr=None, act=None, name=None):
    """Context-window projection per sequence: row t sees rows [t + start, t + start + filter_size) of its own
    sequence (zeros outside), flattened and multiplied by a [filter_size * D, num_filters] filter."""
    from .. import create_parameter
    from ..nn import functional as F

    r = _raw(input)
    off = _offsets(input)
    D = r.shape[1]
    start = -((filter_size - 1) // 2) if padding_start is None else padding_start
    w = create_parameter([filter_size * D, num_filters], r.dtype if r.is_floating_point() else torch.float32,
                         attr=param_attr)
    cols = torch.zeros(r.shape[0], filter_size * D, dtype=r.dtype, device=r.device)
    for a, b in zip(off[:-1], off[1:]):
        for k in range(filter_size):
            sh = start + k
            lo, hi = max(a, a - sh), min(b, b - sh)
            if hi > lo:
                cols[lo:hi, k * D:(k + 1) * D] = r[lo + sh:hi + sh]
    out = cols @ w._t
    if bias_attr is not False:
        bias = create_parameter([num_filters], out.dtype, attr=bias_attr, is_bias=True)
        out = out + bias._t
    res = Tensor._wrap(out)
    if act:
        res = getattr(F, act)(res)
    res._lod = input._lod
    return res


def lod_reset(x, y=None, target_lod=None):
    """New LoD for x: y's LoD (or y's values as offsets) or target_lod offsets."""
    out = Tensor._wrap(_raw(x))
    if y is not None:
        out._lod = getattr(y, "_lod", None) or [[int(v) for v in _raw(y).reshape(-1).tolist()]]
    else:
        out._lod = [list(target_lod)]
    return out


def _install_tensor_lod_methods():
    def set_lod(self, lod):
        self._lod = [list(map(int, lv)) for lv in lod]

    def lod(self):
        return getattr(self, "_lod", None) or []

    def set_recursive_sequence_lengths(self, lens):
        out = []
        for lv in lens:
            o = [0]
            for n in lv:
                o.append(o[-1] + int(n))
            out.append(o)
        self._lod = out

    def recursive_sequence_lengths(self):
        return [[b - a for a, b in zip(lv[:-1], lv[1:])] for lv in self.lod()]

    for n, f in (("set_lod", set_lod), ("lod", lod), ("set_recursive_sequence_lengths",
                                                         set_recursive_sequence_lengths),
                 ("recursive_sequence_lengths", recursive_sequence_lengths)):
        if not hasattr(Tensor, n):
            setattr(Tensor, n, f)


_install_tensor_lod_methods()
