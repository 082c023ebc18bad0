"""Creation ops (reference: python/paddle/tensor/creation.py)."""
from __future__ import annotations

import math

import numpy as np
import torch

from ..framework import dtype as _dt
from ..framework.tensor import Tensor, to_tensor  # noqa: F401
from ._helpers import device, dtype_arg, shape_arg, u, ut, w


def _fdt(dtype):
    return dtype_arg(dtype, _dt.default_float_dtype())


def zeros(shape, dtype=None, name=None):
    return w(torch.zeros(shape_arg(shape), dtype=_fdt(dtype), device=device()))


def ones(shape, dtype=None, name=None):
    return w(torch.ones(shape_arg(shape), dtype=_fdt(dtype), device=device()))


def empty(shape, dtype=None, name=None):
    return w(torch.empty(shape_arg(shape), dtype=_fdt(dtype), device=device()))


def full(shape, fill_value, dtype=None, name=None):
    if isinstance(fill_value, Tensor):
        fill_value = fill_value.item()
    if dtype is None:
        if isinstance(fill_value, bool):
            dt = torch.bool
        elif isinstance(fill_value, int):
            dt = _dt.default_float_dtype()
        else:
            dt = _dt.default_float_dtype()
    else:
        dt = _dt.convert_dtype(dtype)
    return w(torch.full(shape_arg(shape), fill_value, dtype=dt, device=device()))


def zeros_like(x, dtype=None, name=None):
    return w(torch.zeros_like(u(x), dtype=dtype_arg(dtype)))


def ones_like(x, dtype=None, name=None):
    return w(torch.ones_like(u(x), dtype=dtype_arg(dtype)))


def empty_like(x, dtype=None, name=None):
    return w(torch.empty_like(u(x), dtype=dtype_arg(dtype)))


def full_like(x, fill_value, dtype=None, name=None):
    if isinstance(fill_value, Tensor):
        fill_value = fill_value.item()
    return w(torch.full_like(u(x), fill_value, dtype=dtype_arg(dtype)))


def arange(start=0, end=None, step=1, dtype=None, name=None):
    from ._helpers import scalar

    start, end, step = scalar(start), scalar(end), scalar(step)
    if end is None:
        start, end = 0, start
    if dtype is None:
        if all(isinstance(v, (int, np.integer)) for v in (start, end, step)):
            dt = torch.int64
        else:
            dt = _dt.default_float_dtype()
    else:
        dt = _dt.convert_dtype(dtype)
    return w(torch.arange(start, end, step, dtype=dt, device=device()))


def linspace(start, stop, num, dtype=None, name=None):
    from ._helpers import scalar

    return w(torch.linspace(scalar(start), scalar(stop), int(scalar(num)), dtype=_fdt(dtype), device=device()))


def logspace(start, stop, num, base=10.0, dtype=None, name=None):
    from ._helpers import scalar

    return w(torch.logspace(scalar(start), scalar(stop), int(scalar(num)), base=scalar(base), dtype=_fdt(dtype), device=device()))


def eye(num_rows, num_columns=None, dtype=None, name=None):
    num_columns = num_rows if num_columns is None else num_columns
    return w(torch.eye(int(num_rows), int(num_columns), dtype=_fdt(dtype), device=device()))


def diag(x, offset=0, padding_value=0, name=None):
    t = u(x)
    if t.dim() == 1 and padding_value != 0:
        n = t.numel() + abs(offset)
        out = torch.full((n, n), padding_value, dtype=t.dtype, device=t.device)
        return w(out + torch.diag(t, offset) - torch.diag(torch.full_like(t, padding_value), offset))
    return w(torch.diag(t, offset))


def diagflat(x, offset=0, name=None):
    return w(torch.diagflat(u(x), offset))


def diag_embed(input, offset=0, dim1=-2, dim2=-1):
    return w(torch.diag_embed(u(input), offset, dim1, dim2))


def meshgrid(*args, **kwargs):
    if len(args) == 1 and isinstance(args[0], (list, tuple)):
        args = args[0]
    return [w(t) for t in torch.meshgrid(*[u(a) for a in args], indexing="ij")]


def tril(x, diagonal=0, name=None):
    return w(torch.tril(u(x), diagonal))


def triu(x, diagonal=0, name=None):
    return w(torch.triu(u(x), diagonal))


def tril_indices(row, col, offset=0, dtype="int64"):
    return w(torch.tril_indices(row, col, offset, dtype=_dt.convert_dtype(dtype), device=device()))


def triu_indices(row, col=None, offset=0, dtype="int64"):
    col = row if col is None else col
    return w(torch.triu_indices(row, col, offset, dtype=_dt.convert_dtype(dtype), device=device()))


def assign(x, output=None):
    src = ut(x) if not isinstance(x, (list, tuple, np.ndarray)) else to_tensor(x)._t
    if output is None:
        return w(src.clone())
    with torch.no_grad():
        output._t.copy_(src)
    return output


def clone(x, name=None):
    return w(u(x).clone())


def complex(real, imag, name=None):
    return w(torch.complex(u(real), u(imag)))


def polar(abs, angle, name=None):
    return w(torch.polar(u(abs), u(angle)))


def fill_constant(shape, dtype, value, force_cpu=False, out=None, name=None):
    return full(shape, value, dtype)


def create_tensor(dtype, name=None, persistable=False):
    t = w(torch.empty(0, dtype=_dt.convert_dtype(dtype), device=device()))
    t.persistable = persistable
    return t


def cauchy_(x, loc=0, scale=1, name=None):
    with torch.no_grad():
        x._t.cauchy_(loc, scale)
    return x


def geometric_(x, probs, name=None):
    with torch.no_grad():
        x._t.geometric_(probs)
    return x


def vander(x, n=None, increasing=False, name=None):
    return w(torch.linalg.vander(u(x), N=n) if increasing else torch.vander(u(x), N=n))


def _pi():
    return math.pi


__all__ = [_n for _n, _v in list(globals().items())
           if not _n.startswith("_") and callable(_v) and getattr(_v, "__module__", None) == __name__]
