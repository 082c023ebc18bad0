"""paddle.utils (reference: python/paddle/utils/)."""
from __future__ import annotations

import functools
import os
import warnings

from . import cpp_extension, dlpack, unique_name  # noqa: F401


def deprecated(update_to="", since="", reason="", level=0):
    def deco(fn):
        @functools.wraps(fn)
        def inner(*a, **k):
            warnings.warn(f"{fn.__name__} is deprecated since {since}: {reason} {update_to}", DeprecationWarning)
            return fn(*a, **k)

        return inner

    return deco


def try_import(module_name):
    import importlib

    return importlib.import_module(module_name)


def run_check():
    """paddle.utils.run_check: verifies the device, kernels and (multi-device) collectives."""
    import torch

    from .. import to_tensor
    from ..ops import native_available

    x = to_tensor([[1.0, 2.0], [3.0, 4.0]])
    y = (x @ x).sum()
    print(f"paddle2_amd works on {x.place}: result {float(y):.1f}")
    if torch.cuda.is_available():
        print(f"MI355X devices: {torch.cuda.device_count()}, native CDNA4 kernels: {native_available()}")
    print("PaddlePaddle(amd) is installed successfully!")


def flatten(nest):
    out = []
    if isinstance(nest, (list, tuple)):
        for n in nest:
            out.extend(flatten(n))
    elif isinstance(nest, dict):
        for k in sorted(nest):
            out.extend(flatten(nest[k]))
    else:
        out.append(nest)
    return out


def map_structure(func, *structure):
    s0 = structure[0]
    if isinstance(s0, (list, tuple)):
        return type(s0)(map_structure(func, *x) for x in zip(*structure))
    if isinstance(s0, dict):
        return {k: map_structure(func, *[s[k] for s in structure]) for k in s0}
    return func(*structure)
