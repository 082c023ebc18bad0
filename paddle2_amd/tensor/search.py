"""Search / sort ops (reference: python/paddle/tensor/search.py)."""
from __future__ import annotations

import torch

from ..framework import dtype as _dt
from ..framework.tensor import Tensor
from ._helpers import ut

_wrap = Tensor._wrap


def argmax(x, axis=None, keepdim=False, dtype="int64", name=None):
    t = x._t
    if axis is None:
        r = torch.argmax(t.flatten())
        if keepdim:
            r = r.reshape([1] * t.dim())
    else:
        r = torch.argmax(t, dim=int(axis), keepdim=keepdim)
    return _wrap(r.to(_dt.convert_dtype(dtype)))


def argmin(x, axis=None, keepdim=False, dtype="int64", name=None):
    t = x._t
    if axis is None:
        r = torch.argmin(t.flatten())
        if keepdim:
            r = r.reshape([1] * t.dim())
    else:
        r = torch.argmin(t, dim=int(axis), keepdim=keepdim)
    return _wrap(r.to(_dt.convert_dtype(dtype)))


def argsort(x, axis=-1, descending=False, stable=False, name=None):
    return _wrap(torch.argsort(x._t, dim=axis, descending=descending, stable=stable))


def sort(x, axis=-1, descending=False, stable=False, name=None):
    return _wrap(torch.sort(x._t, dim=axis, descending=descending, stable=stable).values)


def topk(x, k, axis=None, largest=True, sorted=True, name=None):
    t = x._t
    k = int(k.item()) if isinstance(k, Tensor) else int(k)
    ax = -1 if axis is None else axis
    v, i = torch.topk(t, k, dim=ax, largest=largest, sorted=sorted)
    return _wrap(v), _wrap(i)


def kthvalue(x, k, axis=None, keepdim=False, name=None):
    ax = -1 if axis is None else axis
    v, i = torch.kthvalue(x._t, k, dim=ax, keepdim=keepdim)
    return _wrap(v), _wrap(i)


def mode(x, axis=-1, keepdim=False, name=None):
    v, i = torch.mode(x._t, dim=axis, keepdim=keepdim)
    return _wrap(v), _wrap(i)


def where(condition, x=None, y=None, name=None):
    c = ut(condition)
    if x is None and y is None:
        return nonzero(condition, as_tuple=True)
    a = ut(x, c if not isinstance(y, Tensor) else y._t)
    b = ut(y, a)
    return _wrap(torch.where(c, a, b))


def where_(condition, x=None, y=None, name=None):
    r = where(condition, x, y)
    with torch.no_grad():
        x._t.copy_(r._t)
    return x


def nonzero(x, as_tuple=False):
    t = x._t
    if as_tuple:
        return tuple(_wrap(i.unsqueeze(-1)) for i in torch.nonzero(t, as_tuple=True))
    return _wrap(torch.nonzero(t))


def masked_select(x, mask, name=None):
    return _wrap(torch.masked_select(x._t, mask._t))


def index_sample(x, index):
    return _wrap(torch.gather(x._t, 1, index._t.long()))


def searchsorted(sorted_sequence, values, out_int32=False, right=False, name=None):
    return _wrap(torch.searchsorted(sorted_sequence._t, values._t, out_int32=out_int32, right=right))


def bucketize(x, sorted_sequence, out_int32=False, right=False, name=None):
    return _wrap(torch.bucketize(x._t, sorted_sequence._t, out_int32=out_int32, right=right))


def top_p_sampling(x, ps, threshold=None, topp_seed=None, seed=-1, k=0, mode="truncated", return_top=False, name=None):
    """Nucleus sampling used by the serving path (reference: phi top_p_sampling kernel)."""
    probs = x._t.float()
    sp, si = torch.sort(probs, dim=-1, descending=True)
    cum = sp.cumsum(-1)
    p = ps._t.float().reshape(-1, 1)
    mask = cum - sp > p
    sp = sp.masked_fill(mask, 0.0)
    sp = sp / sp.sum(-1, keepdim=True)
    g = None
    if seed is not None and seed >= 0:
        g = torch.Generator(device=probs.device).manual_seed(seed)
    choice = torch.multinomial(sp, 1, generator=g)
    ids = si.gather(-1, choice)
    return _wrap(probs.gather(-1, ids).to(x._t.dtype)), _wrap(ids)


__all__ = [_n for _n, _v in list(globals().items())
           if not _n.startswith("_") and callable(_v) and getattr(_v, "__module__", None) == __name__]
