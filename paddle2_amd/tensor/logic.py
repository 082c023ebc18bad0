"""Comparison / logical ops (reference: python/paddle/tensor/logic.py)."""
from __future__ import annotations

import torch

from ..framework.tensor import Tensor
from ._helpers import ut

_wrap = Tensor._wrap


def _cmp(fn):
    def op(x, y, name=None):
        a = ut(x)
        b = y._t if isinstance(y, Tensor) else (y if isinstance(y, (int, float, bool)) else ut(y, a))
        return _wrap(fn(a, b))

    return op


equal = _cmp(torch.eq)
not_equal = _cmp(torch.ne)
less_than = _cmp(torch.lt)
less_equal = _cmp(torch.le)
greater_than = _cmp(torch.gt)
greater_equal = _cmp(torch.ge)
less = less_than
greater = greater_than


def logical_and(x, y, out=None, name=None):
    return _wrap(torch.logical_and(ut(x), ut(y)))


def logical_or(x, y, out=None, name=None):
    return _wrap(torch.logical_or(ut(x), ut(y)))


def logical_xor(x, y, out=None, name=None):
    return _wrap(torch.logical_xor(ut(x), ut(y)))


def equal_all(x, y, name=None):
    a, b = ut(x), ut(y)
    return _wrap(torch.tensor(a.shape == b.shape and bool(torch.equal(a, b)), device=a.device))


def allclose(x, y, rtol=1e-05, atol=1e-08, equal_nan=False, name=None):
    return _wrap(torch.tensor(torch.allclose(ut(x), ut(y), rtol, atol, equal_nan)))


def isclose(x, y, rtol=1e-05, atol=1e-08, equal_nan=False, name=None):
    return _wrap(torch.isclose(ut(x), ut(y), rtol, atol, equal_nan))


def is_tensor(x):
    return isinstance(x, Tensor)


def is_complex(x):
    return x._t.is_complex()


def is_floating_point(x):
    return x._t.is_floating_point()


def is_integer(x):
    t = x._t
    return not (t.is_floating_point() or t.is_complex() or t.dtype == torch.bool)


__all__ = [_n for _n, _v in list(globals().items())
           if not _n.startswith("_") and callable(_v) and getattr(_v, "__module__", None) == __name__]
