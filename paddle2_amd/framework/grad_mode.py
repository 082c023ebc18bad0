"""Grad-mode context managers (python/paddle/base/dygraph/base.py no_grad_ / enable_grad)."""
from __future__ import annotations

import functools

import torch


class no_grad:
    """paddle.no_grad — usable as context manager or decorator."""

    def __enter__(self):
        self._prev = torch.is_grad_enabled()
        torch.set_grad_enabled(False)
        return self

    def __exit__(self, *exc):
        torch.set_grad_enabled(self._prev)
        return False

    def __call__(self, fn):
        @functools.wraps(fn)
        def inner(*a, **k):
            with no_grad():
                return fn(*a, **k)

        return inner


class enable_grad(no_grad):
    def __enter__(self):
        self._prev = torch.is_grad_enabled()
        torch.set_grad_enabled(True)
        return self

    def __call__(self, fn):
        @functools.wraps(fn)
        def inner(*a, **k):
            with enable_grad():
                return fn(*a, **k)

        return inner


class set_grad_enabled:
    def __init__(self, mode: bool):
        self._mode = bool(mode)
        self._prev = torch.is_grad_enabled()
        torch.set_grad_enabled(self._mode)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        torch.set_grad_enabled(self._prev)
        return False


def is_grad_enabled() -> bool:
    return torch.is_grad_enabled()


def in_dynamic_mode() -> bool:
    from ..static import _static_mode_enabled

    return not _static_mode_enabled()
