"""Random ops (reference: python/paddle/tensor/random.py)."""
from __future__ import annotations

import torch

from ..framework import dtype as _dt
from ..framework.tensor import Tensor
from ._helpers import device, dtype_arg, scalar, shape_arg

_wrap = Tensor._wrap


def _fdt(dtype):
    return dtype_arg(dtype, _dt.default_float_dtype())


def _gen(seed):
    if seed:
        g = torch.Generator(device=device())
        g.manual_seed(int(seed))
        return g
    return None


def rand(shape, dtype=None, name=None):
    return _wrap(torch.rand(shape_arg(shape), dtype=_fdt(dtype), device=device()))


def randn(shape, dtype=None, name=None):
    return _wrap(torch.randn(shape_arg(shape), dtype=_fdt(dtype), device=device()))


standard_normal = randn


def randint(low=0, high=None, shape=[1], dtype=None, name=None):
    if high is None:
        low, high = 0, low
    return _wrap(torch.randint(int(low), int(high), shape_arg(shape), dtype=dtype_arg(dtype, torch.int64), device=device()))


def randint_like(x, low=0, high=None, dtype=None, name=None):
    if high is None:
        low, high = 0, low
    return _wrap(torch.randint(int(low), int(high), x.shape, dtype=dtype_arg(dtype, x.dtype), device=x._t.device))


def uniform(shape, dtype=None, min=-1.0, max=1.0, seed=0, name=None):
    t = torch.empty(shape_arg(shape), dtype=_fdt(dtype), device=device())
    t.uniform_(scalar(min), scalar(max), generator=_gen(seed))
    return _wrap(t)


def uniform_(x, min=-1.0, max=1.0, seed=0, name=None):
    with torch.no_grad():
        x._t.uniform_(min, max, generator=_gen(seed))
    return x


def normal(mean=0.0, std=1.0, shape=None, name=None):
    if isinstance(mean, Tensor) or isinstance(std, Tensor):
        m = mean._t if isinstance(mean, Tensor) else torch.tensor(mean, device=device())
        s = std._t if isinstance(std, Tensor) else torch.tensor(std, device=device())
        m, s = torch.broadcast_tensors(m, s)
        return _wrap(torch.normal(m, s))
    return _wrap(torch.normal(float(mean), float(std), shape_arg(shape), device=device(), dtype=_dt.default_float_dtype()))


def normal_(x, mean=0.0, std=1.0, name=None):
    with torch.no_grad():
        x._t.normal_(mean, std)
    return x


def gaussian(shape, mean=0.0, std=1.0, seed=0, dtype=None, name=None):
    t = torch.empty(shape_arg(shape), dtype=_fdt(dtype), device=device())
    t.normal_(mean, std, generator=_gen(seed))
    return _wrap(t)


def randperm(n, dtype="int64", name=None):
    return _wrap(torch.randperm(int(n), dtype=_dt.convert_dtype(dtype), device=device()))


def bernoulli(x, p=None, name=None):
    if p is not None:
        return _wrap(torch.bernoulli(torch.full_like(x._t, p)))
    return _wrap(torch.bernoulli(x._t))


def bernoulli_(x, p=0.5, name=None):
    with torch.no_grad():
        x._t.bernoulli_(p)
    return x


def multinomial(x, num_samples=1, replacement=False, name=None):
    return _wrap(torch.multinomial(x._t, num_samples, replacement))


def poisson(x, name=None):
    return _wrap(torch.poisson(x._t))


def exponential_(x, lam=1.0, name=None):
    with torch.no_grad():
        x._t.exponential_(lam)
    return x


def rand_like(x, dtype=None, name=None):
    return _wrap(torch.rand_like(x._t, dtype=dtype_arg(dtype)))


def randn_like(x, dtype=None, name=None):
    return _wrap(torch.randn_like(x._t, dtype=dtype_arg(dtype)))


def binomial(count, prob, name=None):
    return _wrap(torch.binomial(count._t.float(), prob._t.float()).to(torch.int64))


def standard_gamma(x, name=None):
    return _wrap(torch._standard_gamma(x._t))


__all__ = [_n for _n, _v in list(globals().items())
           if not _n.startswith("_") and callable(_v) and getattr(_v, "__module__", None) == __name__]
