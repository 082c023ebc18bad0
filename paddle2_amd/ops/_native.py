"""Loader for the in-tree native extension ``paddle2_amd._C`` (HIP kernels for gfx950).

Policy: on a machine with an MI355X the native kernels are mandatory — if the extension is
missing we raise instead of silently falling back to ATen (the driver checks which .so files
the GPU tests load).  On CPU-only hosts the ops use their PyTorch reference implementations.
"""
from __future__ import annotations

import importlib
import os

import torch

_C = None
_err = None

DT_CODE = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def _load():
    global _C, _err
    if _C is not None or _err is not None:
        return _C
    if os.environ.get("PADDLE2_AMD_DISABLE_NATIVE") == "1":
        _err = RuntimeError("native kernels disabled by PADDLE2_AMD_DISABLE_NATIVE=1")
        return None
    try:
        _C = importlib.import_module("paddle2_amd._C")
    except Exception as e:  # pragma: no cover - depends on build state
        _err = e
    return _C


def native():
    """Return the extension module or None (CPU hosts / disabled)."""
    return _load()


def available() -> bool:
    return _load() is not None


def require():
    m = _load()
    if m is None:
        raise RuntimeError(
            "paddle2_amd native extension (_C) is not available on a GPU host: build it with "
            "`python -m paddle2_amd._build` (or __graft_entry__.build()). Cause: %r" % (_err,))
    return m


_SYM = []


def _sym_cls():
    if not _SYM:
        from ..static.graph import SymTensor

        _SYM.append(SymTensor)
    return _SYM[0]


def use_native(t: torch.Tensor) -> bool:
    """True when ``t`` lives on the GPU and the kernels must be used.  Symbolic (static-graph recording) tensors
    report the device the Program will run on but have no storage: never hand them to a kernel — the caller's
    composite / graph-op path records them instead."""
    if t.device.type != "cuda" or isinstance(t, _sym_cls()):
        return False
    if os.environ.get("PADDLE2_AMD_DISABLE_NATIVE") == "1":
        return False
    require()
    return True


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()
