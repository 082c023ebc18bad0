"""Static-graph mode switch (full Program/Executor in static/executor.py)."""
from __future__ import annotations

_static = [False]


def _static_mode_enabled():
    return _static[0]


def enable_static():
    _static[0] = True


def disable_static(place=None):
    _static[0] = False


def in_dynamic_mode():
    return not _static[0]


class InputSpec:
    def __init__(self, shape=None, dtype="float32", name=None, stop_gradient=False):
        self.shape = list(shape) if shape is not None else None
        self.dtype = dtype
        self.name = name
        self.stop_gradient = stop_gradient

    @classmethod
    def from_tensor(cls, tensor, name=None):
        return cls(tensor.shape, tensor.dtype, name or tensor.name)

    def __repr__(self):
        return f"InputSpec(shape={self.shape}, dtype={self.dtype}, name={self.name})"
