"""Small shared helpers for the eager op library."""
from __future__ import annotations

import numbers

import numpy as np
import torch

from ..framework import dtype as _dt
from ..framework.place import current_torch_device
from ..framework.tensor import Tensor

_wrap = Tensor._wrap


def u(x):
    if isinstance(x, Tensor):
        return x._t
    if isinstance(x, np.ndarray):
        return torch.from_numpy(np.ascontiguousarray(x)).to(current_torch_device())
    return x


def ut(x, like: torch.Tensor | None = None):
    """Unwrap to a torch tensor (python scalars become tensors on ``like``'s device)."""
    if isinstance(x, Tensor):
        return x._t
    if isinstance(x, torch.Tensor):
        return x
    dev = like.device if like is not None else current_torch_device()
    if isinstance(x, np.ndarray):
        return torch.from_numpy(np.ascontiguousarray(x)).to(dev)
    if isinstance(x, bool):
        return torch.tensor(x, device=dev)
    if isinstance(x, numbers.Integral):
        return torch.tensor(int(x), dtype=torch.int64, device=dev)
    if isinstance(x, numbers.Real):
        return torch.tensor(float(x), dtype=(like.dtype if like is not None and like.is_floating_point() else _dt.default_float_dtype()), device=dev)
    if isinstance(x, (list, tuple)):
        return torch.as_tensor(np.array(x), device=dev)
    raise TypeError(type(x))


def w(t):
    if isinstance(t, torch.Tensor):
        return _wrap(t)
    if isinstance(t, (list, tuple)):
        return [w(x) for x in t] if isinstance(t, list) else tuple(w(x) for x in t)
    return t


def axis_arg(axis):
    if axis is None:
        return None
    if isinstance(axis, Tensor):
        v = axis._t.tolist()
        return tuple(v) if isinstance(v, list) else int(v)
    if isinstance(axis, (list, tuple)):
        if len(axis) == 0:
            return None
        return tuple(int(a.item() if isinstance(a, Tensor) else a) for a in axis)
    return int(axis)


def shape_arg(shape):
    if isinstance(shape, Tensor):
        return [int(s) for s in shape._t.tolist()]
    if isinstance(shape, torch.Size):
        return list(shape)
    if isinstance(shape, (int, np.integer)):
        return [int(shape)]
    return [int(s.item()) if isinstance(s, Tensor) else int(s) for s in shape]


def dtype_arg(dtype, default=None):
    if dtype is None:
        return default
    return _dt.convert_dtype(dtype)


def device():
    return current_torch_device()


def scalar(v):
    if isinstance(v, Tensor):
        return v._t.item()
    return v
