"""InputSpec: the signature of one input of a to_static / jit.save function (reference:
python/paddle/static/input.py ``InputSpec`` — shape with -1/None for dynamic axes, dtype, name,
from_tensor / from_numpy / batch / unbatch)."""
from __future__ import annotations

import numpy as np


def _norm_shape(shape):
    if shape is None:
        return None
    if isinstance(shape, int):
        shape = [shape]
    out = []
    for d in shape:
        if d is None:
            out.append(-1)
        elif isinstance(d, (int, np.integer)):
            if d < -1:
                raise ValueError(f"InputSpec: invalid dimension {d}")
            out.append(int(d))
        else:
            raise TypeError(f"InputSpec: shape entries must be int or None, got {type(d).__name__}")
    return out


def _dtype_name(dtype):
    if dtype is None:
        return "float32"
    s = str(dtype)
    for pre in ("paddle.", "torch.", "paddle2_amd."):
        if s.startswith(pre):
            s = s[len(pre):]
    return s


class InputSpec:
    def __init__(self, shape=None, dtype="float32", name=None, stop_gradient=False):
        self.shape = _norm_shape(shape)
        self.dtype = _dtype_name(dtype)
        self.name = name
        self.stop_gradient = stop_gradient

    @classmethod
    def from_tensor(cls, tensor, name=None):
        return cls(list(tensor.shape), tensor.dtype, name or getattr(tensor, "name", None))

    @classmethod
    def from_numpy(cls, ndarray, name=None):
        return cls(list(ndarray.shape), str(ndarray.dtype), name)

    def batch(self, batch_size):
        """Prepend a batch axis (int, or None / -1 for a dynamic one)."""
        if isinstance(batch_size, (list, tuple)):
            if len(batch_size) != 1:
                raise ValueError("InputSpec.batch takes one batch size")
            batch_size = batch_size[0]
        self.shape = [-1 if batch_size is None else int(batch_size)] + list(self.shape or [])
        return self

    def unbatch(self):
        if not self.shape:
            raise ValueError("InputSpec.unbatch on a spec without axes")
        self.shape = self.shape[1:]
        return self

    def _key(self):
        return (tuple(self.shape) if self.shape is not None else None, self.dtype, self.name, self.stop_gradient)

    def __eq__(self, other):
        return isinstance(other, InputSpec) and self._key() == other._key()

    def __hash__(self):
        return hash(self._key())

    def __repr__(self):
        return f"InputSpec(shape={tuple(self.shape) if self.shape is not None else None}, dtype={self.dtype}, " \
               f"name={self.name}, stop_gradient={self.stop_gradient})"
