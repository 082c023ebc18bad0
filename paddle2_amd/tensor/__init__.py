"""paddle.tensor: the eager op library + Tensor method patching.

Reference: python/paddle/tensor/__init__.py:459 ``tensor_method_func`` — every op below whose
first argument is the tensor is also installed as a ``Tensor`` method.
"""
from __future__ import annotations

import torch

from ..framework.tensor import Tensor, to_tensor
from . import creation, linalg, logic, manipulation, math, random, search, stat
from .creation import *  # noqa: F401,F403
from .linalg import *  # noqa: F401,F403
from .logic import *  # noqa: F401,F403
from .manipulation import *  # noqa: F401,F403
from .math import *  # noqa: F401,F403
from .random import *  # noqa: F401,F403
from .search import *  # noqa: F401,F403
from .stat import *  # noqa: F401,F403
from ._helpers import ut
from . import array  # noqa: E402
from .array import *  # noqa: F401,F403
from . import extra  # noqa: E402
from .extra import *  # noqa: F401,F403
from . import creation, linalg, logic, manipulation, math, random, search, stat  # noqa: F811 (re-bind after star imports)

__all__ = sorted(set(creation.__all__ + linalg.__all__ + logic.__all__ + manipulation.__all__ + math.__all__ +
                     random.__all__ + search.__all__ + stat.__all__ + array.__all__ + extra.__all__ +
                     ["to_tensor", "Tensor"]))

_wrap = Tensor._wrap

# names that must not become methods (creation ops without a tensor first arg etc.)
_NOT_METHODS = {
    "zeros", "ones", "empty", "full", "arange", "linspace", "logspace", "eye", "meshgrid",
    "tril_indices", "triu_indices", "to_tensor", "rand", "randn", "randint", "uniform", "normal",
    "gaussian", "randperm", "standard_normal", "create_tensor", "fill_constant", "complex", "polar",
    "einsum", "concat", "stack", "hstack", "vstack", "dstack", "column_stack", "row_stack",
    "broadcast_tensors", "broadcast_shape", "add_n", "multiplex", "cartesian_prod", "is_tensor",
    "scatter_nd", "multi_dot", "where", "meshgrid", "shape", "rank", "tolist", "block_diag", "log_normal",
}

_METHOD_SOURCES = (math, manipulation, linalg, logic, search, stat, random, creation, extra)


def _install_methods():
    for mod in _METHOD_SOURCES:
        for name in dir(mod):
            if name.startswith("_") or name in _NOT_METHODS:
                continue
            fn = getattr(mod, name)
            mod_name = getattr(fn, "__module__", "") or ""
            if not callable(fn) or isinstance(fn, type) or not mod_name.startswith("paddle2_amd.tensor") \
                    or mod_name.endswith("_helpers"):
                continue
            if name in Tensor.__dict__:
                continue
            setattr(Tensor, name, fn)

    # a few Tensor-method spellings that differ from the functional names
    def _where(self, x=None, y=None, name=None):
        return search.where(self, x, y)

    Tensor.where = _where
    Tensor.mod = math.remainder
    Tensor.floor_mod = math.remainder
    Tensor.matmul = linalg.matmul
    Tensor.tolist = lambda self: self._t.tolist()

    def _reshape_method(self, *shape, name=None):
        if len(shape) == 1 and isinstance(shape[0], (list, tuple, Tensor)):
            shape = shape[0]
        return manipulation.reshape(self, shape)

    Tensor.reshape = _reshape_method
    Tensor.view = manipulation.view
    Tensor.expand = lambda self, *shape, name=None: manipulation.expand(
        self, shape[0] if len(shape) == 1 and isinstance(shape[0], (list, tuple, Tensor)) else shape)
    Tensor.tile = lambda self, *rt, name=None: manipulation.tile(
        self, rt[0] if len(rt) == 1 and isinstance(rt[0], (list, tuple, Tensor)) else rt)
    Tensor.permute = manipulation.permute
    Tensor.cast = lambda self, dtype: manipulation.cast(self, dtype)
    Tensor.cast_ = manipulation.cast_
    Tensor.sum = math.sum
    Tensor.mean = math.mean
    Tensor.max = math.max
    Tensor.min = math.min
    Tensor.abs = math.abs
    Tensor.pow = math.pow
    Tensor.exp = math.exp
    Tensor.sqrt = math.sqrt
    Tensor.all = math.all
    Tensor.any = math.any
    Tensor.split = manipulation.split
    Tensor.chunk = manipulation.chunk
    Tensor.unbind = manipulation.unbind
    Tensor.flatten = manipulation.flatten
    Tensor.squeeze = manipulation.squeeze
    Tensor.unsqueeze = manipulation.unsqueeze
    Tensor.transpose = manipulation.transpose
    Tensor.norm = linalg.norm
    Tensor.numel = lambda self: _wrap(torch.tensor(self._t.numel(), dtype=torch.int64))
    Tensor.equal = logic.equal
    Tensor.uniform_ = random.uniform_
    Tensor.normal_ = random.normal_
    Tensor.exponential_ = random.exponential_
    Tensor.bernoulli_ = random.bernoulli_


def _binop(fn, reverse=False):
    if reverse:
        def op(self, other):
            return fn(other if isinstance(other, Tensor) else _wrap(ut(other, self._t)), self)
    else:
        def op(self, other):
            return fn(self, other)
    return op


def _install_dunders():
    T = Tensor
    T.__add__ = _binop(math.add)
    T.__radd__ = _binop(math.add, True)
    T.__sub__ = _binop(math.subtract)
    T.__rsub__ = lambda self, o: _wrap(ut(o, self._t) - self._t)
    T.__mul__ = _binop(math.multiply)
    T.__rmul__ = _binop(math.multiply, True)
    T.__truediv__ = _binop(math.divide)
    T.__rtruediv__ = lambda self, o: math.divide(_wrap(ut(o, self._t)), self)
    T.__floordiv__ = _binop(math.floor_divide)
    T.__rfloordiv__ = lambda self, o: _wrap(torch.floor_divide(ut(o, self._t), self._t))
    T.__mod__ = _binop(math.remainder)
    T.__rmod__ = lambda self, o: _wrap(torch.remainder(ut(o, self._t), self._t))
    T.__pow__ = _binop(math.pow)
    T.__rpow__ = lambda self, o: _wrap(torch.pow(o if not isinstance(o, Tensor) else o._t, self._t))
    T.__matmul__ = lambda self, o: linalg.matmul(self, o)
    T.__rmatmul__ = lambda self, o: linalg.matmul(o, self)
    T.__neg__ = lambda self: _wrap(-self._t)
    T.__pos__ = lambda self: self
    T.__abs__ = lambda self: _wrap(torch.abs(self._t))
    T.__invert__ = lambda self: _wrap(~self._t)
    T.__and__ = lambda self, o: _wrap(self._t & ut(o, self._t))
    T.__or__ = lambda self, o: _wrap(self._t | ut(o, self._t))
    T.__xor__ = lambda self, o: _wrap(self._t ^ ut(o, self._t))
    T.__rand__ = T.__and__
    T.__ror__ = T.__or__
    T.__rxor__ = T.__xor__
    T.__lshift__ = lambda self, o: _wrap(self._t << ut(o, self._t))
    T.__rshift__ = lambda self, o: _wrap(self._t >> ut(o, self._t))
    T.__eq__ = _binop(logic.equal)
    T.__ne__ = _binop(logic.not_equal)
    T.__lt__ = _binop(logic.less_than)
    T.__le__ = _binop(logic.less_equal)
    T.__gt__ = _binop(logic.greater_than)
    T.__ge__ = _binop(logic.greater_equal)
    T.__hash__ = lambda self: id(self)

    def _iop(tfn):
        def op(self, other):
            o = other._t if isinstance(other, Tensor) else other
            if self._t.requires_grad and self._t.is_leaf:
                self._t = tfn(self._t.clone(), o) if False else getattr(torch, tfn.__name__.rstrip("_"))(self._t, o)
            else:
                tfn(self._t, o)
            return self

        return op

    T.__iadd__ = _iop(torch.Tensor.add_)
    T.__isub__ = _iop(torch.Tensor.sub_)
    T.__imul__ = _iop(torch.Tensor.mul_)
    T.__itruediv__ = _iop(torch.Tensor.div_)


_install_methods()
_install_dunders()
