"""Single-backend op table (the MI355X answer to Phi's KernelFactory).

Reference: phi/core/kernel_factory.h:58 ``KernelKey`` (name, Backend, Layout, DType), :316
``KernelFactory``, :326 ``SelectKernelOrThrowError`` (falls back to CPU); kernel_registry.h:196
``PD_REGISTER_KERNEL``; generated ``_C_ops.<op>`` bindings (python_c_gen.py:113).

Design: there is exactly one device backend (gfx950), so an op is keyed by NAME only.  Each entry
holds the Paddle-signature callable (which itself routes to the hand-written HIP kernel in
``paddle2_amd._C`` when the tensors live on the MI355X, or to its PyTorch reference on CPU), the
dtypes the native kernel covers, and whether a native kernel exists at all.  There is no layout /
backend dimension to search and no multi-backend dispatch; ``select`` is a dict lookup.  The
table is introspectable (``list_ops``, ``kernel_info``) the way ``paddle.base.core`` exposes the
registered kernels, and ``register_op`` is the extension point used by ``paddle.utils.cpp_extension``
style custom ops.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable

import torch


@dataclass
class OpEntry:
    name: str
    fn: Callable
    native_kernel: str | None = None           # symbol in paddle2_amd._C, if a HIP kernel backs it
    dtypes: tuple = (torch.float32, torch.bfloat16, torch.float16)
    inplace: bool = False
    doc: str = ""
    calls: int = field(default=0, compare=False)


_TABLE: dict[str, OpEntry] = {}


def register_op(name, fn=None, *, native_kernel=None, dtypes=None, inplace=False, doc=""):
    """Register ``fn`` under ``name`` (usable as a decorator).  Re-registering replaces the entry."""

    def deco(f):
        _TABLE[name] = OpEntry(name, f, native_kernel, tuple(dtypes) if dtypes else OpEntry.dtypes, inplace,
                               doc or (f.__doc__ or "").strip().split("\n")[0])
        return f

    return deco(fn) if fn is not None else deco


def select(name) -> OpEntry:
    """``SelectKernelOrThrowError`` for a single backend: lookup or a typed error."""
    e = _TABLE.get(name)
    if e is None:
        from .op_schema import NATIVE, resolve

        fn = resolve(name)
        if fn is not None:
            register_op(name, fn, native_kernel=NATIVE.get(name), inplace=name.endswith("_"))
            e = _TABLE[name]
    if e is None:
        raise NotImplementedError(f"op '{name}' is not registered in the paddle2_amd op table "
                                  f"({len(_TABLE)} ops registered)")
    return e


def call(name, *args, **kwargs):
    e = select(name)
    e.calls += 1
    return e.fn(*args, **kwargs)


def has_op(name) -> bool:
    return name in _TABLE


def list_ops(populate=True):
    """Registered op names; by default the whole resolvable reference inventory (ops/op_schema.py)."""
    if populate:
        from .op_schema import _POPULATED, populate as _populate

        if not _POPULATED[0]:
            _populate()
    return sorted(_TABLE)


def kernel_info(name) -> dict:
    """Which implementation runs for ``name`` on this host."""
    from . import _native

    e = select(name)
    native = e.native_kernel is not None and _native.available() and hasattr(_native.native(), e.native_kernel)
    return {"name": name, "native_kernel": e.native_kernel, "native_loaded": bool(native),
            "dtypes": [str(d).replace("torch.", "") for d in e.dtypes], "inplace": e.inplace, "doc": e.doc}


def call_counts():
    return {k: v.calls for k, v in _TABLE.items() if v.calls}
