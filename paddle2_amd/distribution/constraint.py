"""Constraints on distribution parameters and values (reference: python/paddle/distribution/constraint.py).

A constraint is a callable returning an elementwise boolean tensor: does ``value`` lie in the set?  The random-
variable domains (``variable.py``) and the transforms' domain / codomain checks use them; ``real``, ``positive``
and ``simplex`` are the shared singletons.
"""
from __future__ import annotations

import torch

from .distribution import _wrap, raw

__all__ = ["Constraint", "Range", "Real", "Positive", "Simplex", "real", "positive", "simplex"]


class Constraint:
    def __call__(self, value):
        raise NotImplementedError


class _Real(Constraint):
    def __call__(self, value):
        v = raw(value)
        return _wrap(v == v)


class Range(Constraint):
    def __init__(self, lower, upper):
        self._lower, self._upper = lower, upper

    def __call__(self, value):
        v = raw(value)
        return _wrap((raw(self._lower) <= v) & (v <= raw(self._upper)))


class _Positive(Constraint):
    def __call__(self, value):
        return _wrap(raw(value) >= 0.0)


class _Simplex(Constraint):
    def __call__(self, value):
        v = raw(value)
        return _wrap(torch.all(v >= 0, dim=-1) & ((v.sum(-1) - 1).abs() < 1e-6))


real = _Real()
positive = _Positive()
simplex = _Simplex()


# public names as in the reference module
Real = _Real
Positive = _Positive
Simplex = _Simplex
