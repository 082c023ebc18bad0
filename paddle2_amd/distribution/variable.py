"""Random-variable domains (reference: python/paddle/distribution/variable.py); the constraints they check are in
constraint.py."""
from __future__ import annotations

import torch

from .constraint import Constraint, Range, _Positive, _Real, _Simplex, positive, real, simplex  # noqa: F401
from .distribution import _wrap, raw


class Variable:
    """A random variable's domain: discreteness, event rank and its constraint."""

    def __init__(self, is_discrete=False, event_rank=0, constraint=None):
        self._is_discrete = is_discrete
        self._event_rank = event_rank
        self._constraint = constraint

    @property
    def is_discrete(self):
        return self._is_discrete

    @property
    def event_rank(self):
        return self._event_rank

    def constraint(self, value):
        return self._constraint(value)


class Real(Variable):
    def __init__(self, event_rank=0):
        super().__init__(False, event_rank, real)


class Positive(Variable):
    def __init__(self, event_rank=0):
        super().__init__(False, event_rank, positive)


class Independent(Variable):
    """Reinterprets the rightmost ``reinterpreted_batch_rank`` batch axes of ``base`` as event axes."""

    def __init__(self, base, reinterpreted_batch_rank):
        self._base = base
        self._reinterpreted_batch_rank = reinterpreted_batch_rank
        super().__init__(base.is_discrete, base.event_rank + reinterpreted_batch_rank)

    def constraint(self, value):
        ret = raw(self._base.constraint(value))
        if ret.dim() < self._reinterpreted_batch_rank:
            raise ValueError(f"Input dimensions must be equal or grater than {self._reinterpreted_batch_rank}")
        return _wrap(ret.reshape(ret.shape[:ret.dim() - self._reinterpreted_batch_rank] + (-1,)).all(-1))


class Stack(Variable):
    def __init__(self, vars, axis=0):
        self._vars = list(vars)
        self._axis = axis
        super().__init__()

    @property
    def is_discrete(self):
        return any(v.is_discrete for v in self._vars)

    @property
    def event_rank(self):
        rank = max(v.event_rank for v in self._vars)
        if self._axis + rank < 0:
            rank += 1
        return rank

    def constraint(self, value):
        v = raw(value)
        if not (-v.dim() <= self._axis < v.dim()):
            raise ValueError(f"Input dimensions {v.dim()} should be grater than stack constraint axis {self._axis}.")
        parts = [raw(var.constraint(_wrap(x))) for var, x in zip(self._vars, torch.unbind(v, self._axis))]
        return _wrap(torch.stack(parts, self._axis))
