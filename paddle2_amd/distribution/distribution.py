"""Distribution base class (reference: python/paddle/distribution/distribution.py).

Parameters are held as framework Tensors (so gradients flow to them from ``log_prob`` / ``rsample`` /
``entropy``); the math runs on their torch storage through the helpers below and results come back wrapped.
Python numbers / lists / numpy arrays are converted to float32 Tensors and broadcast against each other, as
the reference's ``_to_tensor`` does.
"""
from __future__ import annotations

import math
import numbers
import warnings

import numpy as np
import torch

from ..framework.tensor import Tensor

_wrap = Tensor._wrap


def raw(x, dtype=None):
    """framework Tensor / number / array -> torch tensor (keeps autograd history of Tensors)."""
    if isinstance(x, Tensor):
        t = x._t
    elif isinstance(x, torch.Tensor):
        t = x
    else:
        a = np.asarray(x)
        if a.dtype == np.float64 and dtype is None:
            a = a.astype(np.float32)
        t = torch.as_tensor(a)
        if not t.is_floating_point() and not t.is_complex() and dtype is None:
            t = t.to(torch.float32)
    return t.to(dtype) if dtype is not None and t.dtype != dtype else t


def params(*args):
    """Convert distribution parameters: Tensors pass through; numbers/lists/arrays become float32 Tensors
    broadcast to their common shape (reference Distribution._to_tensor)."""
    if all(isinstance(a, Tensor) for a in args):
        return tuple(args)
    if any(isinstance(a, Tensor) for a in args):
        ts = [raw(a) for a in args]
        dt = next(t.dtype for a, t in zip(args, ts) if isinstance(a, Tensor))
        dev = next(t.device for a, t in zip(args, ts) if isinstance(a, Tensor))
        return tuple(a if isinstance(a, Tensor) else _wrap(t.to(dt).to(dev)) for a, t in zip(args, ts))
    arrs = [np.asarray(a) for a in args]
    dt = np.float64 if all(a.dtype == np.float64 and not isinstance(x, (float, list, tuple))
                           for a, x in zip(arrs, args)) else np.float32
    shape = np.broadcast_shapes(*[a.shape for a in arrs])
    return tuple(_wrap(torch.as_tensor(np.broadcast_to(a.astype(dt), shape).copy())) for a in arrs)


def value_like(param, value):
    """Cast ``value`` to the parameter dtype (reference _check_values_dtype_in_probs)."""
    v = raw(value)
    p = raw(param)
    if v.dtype != p.dtype and (v.is_floating_point() or not p.is_floating_point()):
        if v.is_floating_point():
            warnings.warn("dtype of input 'value' needs to be the same as parameters of distribution class. "
                          "dtype of 'value' will be converted.")
        v = v.to(p.dtype)
    elif v.dtype != p.dtype:
        v = v.to(p.dtype)
    return v.to(p.device)


def sum_rightmost(t, n):
    return t.sum(dim=list(range(-n, 0))) if n > 0 else t


class Distribution:
    """Abstract base: ``batch_shape`` (independent, non-identical draws) and ``event_shape`` (one draw)."""

    def __init__(self, batch_shape=(), event_shape=()):
        self._batch_shape = tuple(batch_shape)
        self._event_shape = tuple(event_shape)

    @property
    def batch_shape(self):
        return self._batch_shape

    @property
    def event_shape(self):
        return self._event_shape

    @property
    def mean(self):
        raise NotImplementedError

    @property
    def variance(self):
        raise NotImplementedError

    @property
    def stddev(self):
        return _wrap(raw(self.variance).sqrt())

    def sample(self, shape=()):
        raise NotImplementedError

    def rsample(self, shape=()):
        raise NotImplementedError

    def entropy(self):
        raise NotImplementedError

    def kl_divergence(self, other):
        from .kl import kl_divergence

        return kl_divergence(self, other)

    def prob(self, value):
        return _wrap(raw(self.log_prob(value)).exp())

    def log_prob(self, value):
        raise NotImplementedError

    def probs(self, value):
        return self.prob(value)

    def _extend_shape(self, sample_shape):
        return tuple(int(s) for s in sample_shape) + tuple(self._batch_shape) + tuple(self._event_shape)

    def _validate_args(self, *args):
        is_t = [isinstance(a, Tensor) for a in args]
        if any(is_t) and not all(is_t):
            raise ValueError("if one argument is Tensor, all arguments should be Tensor")
        return all(is_t) and bool(args)

    def _to_tensor(self, *args):
        return params(*args)

    def _check_values_dtype_in_probs(self, param, value):
        return _wrap(value_like(param, value))

    def _probs_to_logits(self, probs, is_binary=False):
        p = raw(probs)
        return _wrap(p.log() - torch.log1p(-p) if is_binary else p.log())

    def _logits_to_probs(self, logits, is_binary=False):
        lg = raw(logits)
        return _wrap(torch.sigmoid(lg) if is_binary else torch.softmax(lg, dim=-1))

    def __repr__(self):
        return f"{type(self).__name__}(batch_shape={list(self._batch_shape)}, event_shape={list(self._event_shape)})"


def check_shape(shape):
    if not isinstance(shape, (list, tuple)) and not (hasattr(shape, "__iter__")):
        raise TypeError("sample shape must be Iterable object.")
    return [int(s) for s in shape]


def is_number(x):
    return isinstance(x, numbers.Real) and not isinstance(x, bool)


EULER = 0.57721566490153286060
LOG_2PI = math.log(2 * math.pi)
