"""Loader for the host-only native runtime ``paddle2_amd._runtime`` (TCPStore, comm watchdog, host
tracer, blocking queue).  Built on first use if the in-tree .so is missing (g++ only, ~10 s)."""
from __future__ import annotations

_mod = None


def get():
    global _mod
    if _mod is None:
        try:
            from . import _runtime as m
        except ImportError:
            from . import _build

            _build.build_runtime()
            import importlib

            m = importlib.import_module("paddle2_amd._runtime")
        _mod = m
    return _mod
