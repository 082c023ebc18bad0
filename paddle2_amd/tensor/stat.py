"""Statistics (reference: python/paddle/tensor/stat.py)."""
from __future__ import annotations

import torch

from ..framework.tensor import Tensor
from ._helpers import axis_arg

_wrap = Tensor._wrap


def std(x, axis=None, unbiased=True, keepdim=False, name=None):
    ax = axis_arg(axis)
    return _wrap(torch.std(x._t, dim=ax, unbiased=unbiased, keepdim=keepdim))


def var(x, axis=None, unbiased=True, keepdim=False, name=None):
    ax = axis_arg(axis)
    return _wrap(torch.var(x._t, dim=ax, unbiased=unbiased, keepdim=keepdim))


def median(x, axis=None, keepdim=False, mode="avg", name=None):
    t = x._t
    if axis is None:
        t = t.flatten()
        ax = 0
    else:
        ax = int(axis)
    if mode == "avg":
        r = torch.quantile(t.float() if not t.is_floating_point() else t, 0.5, dim=ax, keepdim=keepdim)
        if axis is None and keepdim:
            r = r.reshape([1] * x._t.dim())
        return _wrap(r)
    v, i = torch.median(t, dim=ax, keepdim=keepdim)
    return _wrap(v), _wrap(i)


def nanmedian(x, axis=None, keepdim=False, mode="avg", name=None):
    t = x._t
    if axis is None:
        return _wrap(torch.nanquantile(t.flatten(), 0.5))
    return _wrap(torch.nanquantile(t, 0.5, dim=int(axis), keepdim=keepdim))


def quantile(x, q, axis=None, keepdim=False, interpolation="linear", name=None):
    t = x._t
    qq = q._t if isinstance(q, Tensor) else torch.as_tensor(q, dtype=t.dtype, device=t.device)
    if axis is None:
        return _wrap(torch.quantile(t.flatten(), qq, interpolation=interpolation))
    if isinstance(axis, (list, tuple)):
        dims = sorted(a % t.dim() for a in axis)
        perm = [d for d in range(t.dim()) if d not in dims] + dims
        t2 = t.permute(perm).flatten(len(perm) - len(dims))
        r = torch.quantile(t2, qq, dim=-1, interpolation=interpolation)
        if keepdim:
            for d in dims:
                r = r.unsqueeze(d if qq.dim() == 0 else d + 1)
        return _wrap(r)
    return _wrap(torch.quantile(t, qq, dim=int(axis), keepdim=keepdim, interpolation=interpolation))


def nanquantile(x, q, axis=None, keepdim=False, interpolation="linear", name=None):
    t = x._t
    qq = q._t if isinstance(q, Tensor) else torch.as_tensor(q, dtype=t.dtype, device=t.device)
    if axis is None:
        return _wrap(torch.nanquantile(t.flatten(), qq, interpolation=interpolation))
    return _wrap(torch.nanquantile(t, qq, dim=int(axis), keepdim=keepdim, interpolation=interpolation))


__all__ = [_n for _n, _v in list(globals().items())
           if not _n.startswith("_") and callable(_v) and getattr(_v, "__module__", None) == __name__]
