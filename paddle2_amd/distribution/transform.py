"""Bijective / injective transforms of random variables (reference: python/paddle/distribution/transform.py).

Every transform implements ``_forward`` / ``_inverse`` / ``_forward_log_det_jacobian`` on torch tensors; the
public ``forward`` / ``inverse`` / ``*_log_det_jacobian`` take and return framework Tensors.  A missing
log-det-Jacobian direction is derived from the other one (``ildj(y) = -fldj(inverse(y))``).
"""
from __future__ import annotations

import enum
import functools
import math
import operator

import torch
import torch.nn.functional as F

from . import variable
from .distribution import Distribution, _wrap, raw, sum_rightmost

__all__ = ["Transform", "AbsTransform", "AffineTransform", "ChainTransform", "ExpTransform", "IndependentTransform",
           "PowerTransform", "ReshapeTransform", "SigmoidTransform", "SoftmaxTransform", "StackTransform",
           "StickBreakingTransform", "TanhTransform"]


class Type(enum.Enum):
    BIJECTION = "bijection"
    INJECTION = "injection"
    SURJECTION = "surjection"
    OTHER = "other"

    @classmethod
    def is_injective(cls, _type):
        return _type in (cls.BIJECTION, cls.INJECTION)


def _w(x):
    if isinstance(x, tuple):
        return tuple(_w(v) for v in x)
    return _wrap(x) if isinstance(x, torch.Tensor) else x


def _r(x):
    if isinstance(x, tuple):
        return tuple(_r(v) for v in x)
    return raw(x)


class Transform:
    _type = Type.INJECTION

    def __init__(self):
        super().__init__()

    @classmethod
    def _is_injective(cls):
        return Type.is_injective(cls._type)

    def __call__(self, input):
        from .transformed_distribution import TransformedDistribution

        if isinstance(input, Distribution):
            return TransformedDistribution(input, [self])
        if isinstance(input, Transform):
            return ChainTransform([self, input])
        return self.forward(input)

    def _check_rank(self, x, dom):
        t = raw(x)
        if t.dim() < dom.event_rank:
            raise ValueError(f"The dimensions of x({t.dim()}) should be grater than or equal to "
                             f"{dom.event_rank}")

    def forward(self, x):
        self._check_rank(x, self._domain)
        return _w(self._forward(raw(x)))

    def inverse(self, y):
        self._check_rank(y, self._codomain)
        return _w(self._inverse(raw(y)))

    def forward_log_det_jacobian(self, x):
        self._check_rank(x, self._domain)
        if not self._is_injective():
            raise NotImplementedError("forward_log_det_jacobian can't be implemented for non-injective transforms.")
        return _w(self._call_fldj(raw(x)))

    def inverse_log_det_jacobian(self, y):
        self._check_rank(y, self._codomain)
        return _w(self._call_ildj(raw(y)))

    def forward_shape(self, shape):
        return self._forward_shape(tuple(shape))

    def inverse_shape(self, shape):
        return self._inverse_shape(tuple(shape))

    @property
    def _domain(self):
        return variable.Real()

    @property
    def _codomain(self):
        return variable.Real()

    def _forward(self, x):
        raise NotImplementedError

    def _inverse(self, y):
        raise NotImplementedError

    def _call_fldj(self, x):
        if type(self)._forward_log_det_jacobian is not Transform._forward_log_det_jacobian:
            return self._forward_log_det_jacobian(x)
        if type(self)._inverse_log_det_jacobian is not Transform._inverse_log_det_jacobian:
            return -self._inverse_log_det_jacobian(self._forward(x))
        raise NotImplementedError(f"{type(self).__name__} defines neither log-det-Jacobian direction")

    def _call_ildj(self, y):
        if type(self)._inverse_log_det_jacobian is not Transform._inverse_log_det_jacobian:
            return self._inverse_log_det_jacobian(y)
        if type(self)._forward_log_det_jacobian is not Transform._forward_log_det_jacobian:
            return -self._forward_log_det_jacobian(self._inverse(y))
        raise NotImplementedError(f"{type(self).__name__} defines neither log-det-Jacobian direction")

    def _forward_log_det_jacobian(self, x):
        raise NotImplementedError

    def _inverse_log_det_jacobian(self, y):
        raise NotImplementedError

    def _forward_shape(self, shape):
        return shape

    def _inverse_shape(self, shape):
        return shape


class AbsTransform(Transform):
    """y = |x| (surjective: the inverse returns both pre-images)."""

    _type = Type.SURJECTION

    def _forward(self, x):
        return x.abs()

    def _inverse(self, y):
        return -y, y

    def _inverse_log_det_jacobian(self, y):
        zero = torch.zeros((), dtype=y.dtype, device=y.device)
        return zero, zero

    def inverse_log_det_jacobian(self, y):
        return _w(self._inverse_log_det_jacobian(raw(y)))

    @property
    def _codomain(self):
        return variable.Positive()


class AffineTransform(Transform):
    """y = loc + scale * x."""

    _type = Type.BIJECTION

    def __init__(self, loc, scale):
        from ..framework.tensor import Tensor

        if not isinstance(loc, Tensor):
            raise TypeError(f"Expected 'loc' is a Tensor, but got {type(loc)}")
        if not isinstance(scale, Tensor):
            raise TypeError(f"Expected scale is a Tensor, but got {type(scale)}")
        self._loc, self._scale = loc, scale
        super().__init__()

    @property
    def loc(self):
        return self._loc

    @property
    def scale(self):
        return self._scale

    def _forward(self, x):
        return raw(self._loc) + raw(self._scale) * x

    def _inverse(self, y):
        return (y - raw(self._loc)) / raw(self._scale)

    def _forward_log_det_jacobian(self, x):
        return raw(self._scale).abs().log()

    def _forward_shape(self, shape):
        return tuple(torch.broadcast_shapes(shape, tuple(raw(self._loc).shape), tuple(raw(self._scale).shape)))

    _inverse_shape = _forward_shape


class ChainTransform(Transform):
    """Composition: x -> transforms[0] -> transforms[1] -> ..."""

    def __init__(self, transforms):
        if not isinstance(transforms, (list, tuple)):
            raise TypeError(f"Type of transforms is invalid, expected Sequence, but got {type(transforms)}")
        if not all(isinstance(t, Transform) for t in transforms):
            raise TypeError("All elements of transforms should be Transform type.")
        self.transforms = list(transforms)
        super().__init__()

    def _is_injective(self):
        return all(t._is_injective() for t in self.transforms)

    def _forward(self, x):
        for t in self.transforms:
            x = t._forward(x)
        return x

    def _inverse(self, y):
        for t in reversed(self.transforms):
            y = t._inverse(y)
        return y

    def _forward_log_det_jacobian(self, x):
        value = 0.0
        event_rank = self._domain.event_rank
        for t in self.transforms:
            value = value + sum_rightmost(t._call_fldj(x), event_rank - t._domain.event_rank)
            x = t._forward(x)
            event_rank += t._codomain.event_rank - t._domain.event_rank
        return value

    def _forward_shape(self, shape):
        for t in self.transforms:
            shape = t._forward_shape(shape)
        return shape

    def _inverse_shape(self, shape):
        for t in reversed(self.transforms):
            shape = t._inverse_shape(shape)
        return shape

    def _event_ranks(self):
        """(input, output) event rank of the chain.  Stage i is defined on ``dom_i`` event dims and changes the
        rank by ``shift_i``; at the chain input it therefore needs ``dom_i - (shifts before i)`` dims, and the
        last stage's output needs ``cod_last - (all shifts)``.  The chain takes the largest requirement; the
        output rank is the input rank plus every shift."""
        shifts = [t._codomain.event_rank - t._domain.event_rank for t in self.transforms]
        needs, acc = [], 0
        for t, sh in zip(self.transforms, shifts):
            needs.append(t._domain.event_rank - acc)
            acc += sh
        needs.append(self.transforms[-1]._codomain.event_rank - acc)
        r_in = max(needs)
        return r_in, r_in + acc

    @property
    def _domain(self):
        if not self.transforms:
            return variable.Real()
        base = self.transforms[0]._domain
        return variable.Independent(base, self._event_ranks()[0] - base.event_rank)

    @property
    def _codomain(self):
        if not self.transforms:
            return variable.Real()
        base = self.transforms[-1]._codomain
        return variable.Independent(base, self._event_ranks()[1] - base.event_rank)


class ExpTransform(Transform):
    _type = Type.BIJECTION

    @property
    def _codomain(self):
        return variable.Positive()

    def _forward(self, x):
        return x.exp()

    def _inverse(self, y):
        return y.log()

    def _forward_log_det_jacobian(self, x):
        return x


class IndependentTransform(Transform):
    """Treat the rightmost ``reinterpreted_batch_rank`` batch axes of ``base``'s input as event axes."""

    def __init__(self, base, reinterpreted_batch_rank):
        if not isinstance(base, Transform):
            raise TypeError(f"Expected 'base' is Transform type, but get {type(base)}")
        if reinterpreted_batch_rank <= 0:
            raise ValueError(f"Expected 'reinterpreted_batch_rank' is grater than zero, but got "
                             f"{reinterpreted_batch_rank}")
        self._base = base
        self._reinterpreted_batch_rank = reinterpreted_batch_rank
        super().__init__()

    def _is_injective(self):
        return self._base._is_injective()

    def _forward(self, x):
        return self._base._forward(x)

    def _inverse(self, y):
        return self._base._inverse(y)

    def _forward_log_det_jacobian(self, x):
        return sum_rightmost(self._base._call_fldj(x), self._reinterpreted_batch_rank)

    def _forward_shape(self, shape):
        return self._base._forward_shape(shape)

    def _inverse_shape(self, shape):
        return self._base._inverse_shape(shape)

    @property
    def _domain(self):
        return variable.Independent(self._base._domain, self._reinterpreted_batch_rank)

    @property
    def _codomain(self):
        return variable.Independent(self._base._codomain, self._reinterpreted_batch_rank)


class PowerTransform(Transform):
    """y = x ** power."""

    _type = Type.BIJECTION

    def __init__(self, power):
        from ..framework.tensor import Tensor

        if not isinstance(power, Tensor):
            raise TypeError(f"Expected 'power' is a tensor, but got {type(power)}")
        self._power = power
        super().__init__()

    @property
    def power(self):
        return self._power

    @property
    def _codomain(self):
        return variable.Positive()

    def _forward(self, x):
        return x.pow(raw(self._power))

    def _inverse(self, y):
        return y.pow(1 / raw(self._power))

    def _forward_log_det_jacobian(self, x):
        p = raw(self._power)
        return (p * x.pow(p - 1)).abs().log()

    def _forward_shape(self, shape):
        return tuple(torch.broadcast_shapes(shape, tuple(raw(self._power).shape)))

    _inverse_shape = _forward_shape


class ReshapeTransform(Transform):
    """Reshape the event part: in_event_shape -> out_event_shape (same number of elements)."""

    _type = Type.BIJECTION

    def __init__(self, in_event_shape, out_event_shape):
        if not isinstance(in_event_shape, (list, tuple)) or not isinstance(out_event_shape, (list, tuple)):
            raise TypeError(f"Expected type of 'in_event_shape' and 'out_event_shape' is Sequence[int], but got "
                            f"'in_event_shape': {in_event_shape}, 'out_event_shape': {out_event_shape}")
        prod = lambda s: functools.reduce(operator.mul, s, 1)  # noqa: E731
        if prod(in_event_shape) != prod(out_event_shape):
            raise ValueError(f"The numel of 'in_event_shape' should be 'out_event_shape', but got "
                             f"{prod(in_event_shape)}!={prod(out_event_shape)}")
        self._in_event_shape = tuple(in_event_shape)
        self._out_event_shape = tuple(out_event_shape)
        super().__init__()

    @property
    def in_event_shape(self):
        return self._in_event_shape

    @property
    def out_event_shape(self):
        return self._out_event_shape

    @property
    def _domain(self):
        return variable.Independent(variable.Real(), len(self._in_event_shape))

    @property
    def _codomain(self):
        return variable.Independent(variable.Real(), len(self._out_event_shape))

    def _forward(self, x):
        return x.reshape(tuple(x.shape)[:x.dim() - len(self._in_event_shape)] + self._out_event_shape)

    def _inverse(self, y):
        return y.reshape(tuple(y.shape)[:y.dim() - len(self._out_event_shape)] + self._in_event_shape)

    def _forward_shape(self, shape):
        n = len(self._in_event_shape)
        if len(shape) < n or tuple(shape[len(shape) - n:]) != self._in_event_shape:
            raise ValueError(f"Event shape mismatch, expected: {self._in_event_shape}, but got "
                             f"{tuple(shape[len(shape) - n:])}")
        return tuple(shape[:len(shape) - n]) + self._out_event_shape

    def _inverse_shape(self, shape):
        n = len(self._out_event_shape)
        if len(shape) < n or tuple(shape[len(shape) - n:]) != self._out_event_shape:
            raise ValueError(f"Event shape mismatch, expected: {self._out_event_shape}, but got "
                             f"{tuple(shape[len(shape) - n:])}")
        return tuple(shape[:len(shape) - n]) + self._in_event_shape

    def _forward_log_det_jacobian(self, x):
        return torch.zeros(tuple(x.shape)[:x.dim() - len(self._in_event_shape)], dtype=x.dtype, device=x.device)


class SigmoidTransform(Transform):
    _type = Type.BIJECTION

    @property
    def _codomain(self):
        return variable.Variable(False, 0, variable.Range(0.0, 1.0))

    def _forward(self, x):
        return torch.sigmoid(x)

    def _inverse(self, y):
        return y.log() - torch.log1p(-y)

    def _forward_log_det_jacobian(self, x):
        return -F.softplus(-x) - F.softplus(x)


class SoftmaxTransform(Transform):
    """Unconstrained vector -> simplex (not injective: no log-det-Jacobian)."""

    _type = Type.OTHER

    @property
    def _domain(self):
        return variable.Independent(variable.Real(), 1)

    @property
    def _codomain(self):
        return variable.Variable(False, 1, variable.simplex)

    def _forward(self, x):
        e = (x - x.amax(-1, keepdim=True)).exp()
        return e / e.sum(-1, keepdim=True)

    def _inverse(self, y):
        return y.log()

    def _forward_shape(self, shape):
        if len(shape) < 1:
            raise ValueError(f"Expected length of shape is grater than 1, but got {len(shape)}")
        return shape

    _inverse_shape = _forward_shape


class StackTransform(Transform):
    """Apply ``transforms[i]`` to slice i along ``axis``."""

    def __init__(self, transforms, axis=0):
        if not transforms or not isinstance(transforms, (list, tuple)):
            raise TypeError(f"Expected 'transforms' is Sequence[Transform], but got {type(transforms)}.")
        if not all(isinstance(t, Transform) for t in transforms):
            raise TypeError("Expected all element in transforms is Transform Type.")
        if not isinstance(axis, int):
            raise TypeError(f"Expected 'axis' is int, but got{type(axis)}.")
        self._transforms = list(transforms)
        self._axis = axis
        super().__init__()

    def _is_injective(self):
        return all(t._is_injective() for t in self._transforms)

    @property
    def transforms(self):
        return self._transforms

    @property
    def axis(self):
        return self._axis

    def _check_size(self, v):
        if not (-v.dim() <= self._axis < v.dim()):
            raise ValueError(f"Input dimensions {v.dim()} should be grater than stack transform axis {self._axis}.")
        if v.shape[self._axis] != len(self._transforms):
            raise ValueError(f"Input size along {self._axis} should be equal to the length of transforms.")

    def _map(self, v, fn):
        self._check_size(v)
        return torch.stack([fn(t, x) for t, x in zip(self._transforms, torch.unbind(v, self._axis))], self._axis)

    def _forward(self, x):
        return self._map(x, lambda t, v: t._forward(v))

    def _inverse(self, y):
        return self._map(y, lambda t, v: t._inverse(v))

    def _forward_log_det_jacobian(self, x):
        return self._map(x, lambda t, v: t._call_fldj(v))

    @property
    def _domain(self):
        return variable.Stack([t._domain for t in self._transforms], self._axis)

    @property
    def _codomain(self):
        return variable.Stack([t._codomain for t in self._transforms], self._axis)


class StickBreakingTransform(Transform):
    """Unconstrained R^K -> simplex in R^(K+1) by stick breaking."""

    _type = Type.BIJECTION

    def _forward(self, x):
        offset = x.shape[-1] + 1 - torch.ones_like(x).cumsum(-1)
        z = torch.sigmoid(x - offset.log())
        zc = (1 - z).cumprod(-1)
        return F.pad(z, [0, 1], value=1.0) * F.pad(zc, [1, 0], value=1.0)

    def _inverse(self, y):
        yc = y[..., :-1]
        offset = y.shape[-1] - torch.ones_like(yc).cumsum(-1)
        sf = 1 - yc.cumsum(-1)
        return yc.log() - sf.log() + offset.log()

    def _forward_log_det_jacobian(self, x):
        y = self._forward(x)
        offset = x.shape[-1] + 1 - torch.ones_like(x).cumsum(-1)
        x = x - offset.log()
        return (-x + F.logsigmoid(x) + y[..., :-1].log()).sum(-1)

    def _forward_shape(self, shape):
        if not shape:
            raise ValueError(f"Expected 'shape' is not empty, but got {shape}")
        return tuple(shape[:-1]) + (shape[-1] + 1,)

    def _inverse_shape(self, shape):
        if not shape:
            raise ValueError(f"Expected 'shape' is not empty, but got {shape}")
        return tuple(shape[:-1]) + (shape[-1] - 1,)

    @property
    def _domain(self):
        return variable.Independent(variable.Real(), 1)

    @property
    def _codomain(self):
        return variable.Variable(False, 1, variable.simplex)


class TanhTransform(Transform):
    _type = Type.BIJECTION

    @property
    def _codomain(self):
        return variable.Variable(False, 0, variable.Range(-1.0, 1.0))

    def _forward(self, x):
        return x.tanh()

    def _inverse(self, y):
        return torch.atanh(y)

    def _forward_log_det_jacobian(self, x):
        # log(1 - tanh(x)^2) in a form stable for large |x|
        return 2.0 * (math.log(2.0) - x - F.softplus(-2.0 * x))
