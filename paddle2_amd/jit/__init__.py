"""paddle.jit (reference: python/paddle/jit/api.py ``to_static`` / ``save`` / ``load``,
dy2static ``StaticFunction`` / ``TranslatedLayer``).

``to_static`` converts a Layer or function into a static Program per input signature: the first
call with a new (shapes, dtypes) signature records the Program by running the dygraph code on
symbolic inputs (paddle2_amd.static.graph — Python control flow is resolved at record time, the
same contract as the reference's tracing mode), later calls replay it through the Executor; with
``build_strategy.enable_cuda_graph`` the replay is a HIP graph launch.  Outputs are ordinary
tensors with autograd history, so a to_static layer still trains.  ``save`` writes the inference
Program (``.pdmodel``) + parameters (``.pdiparams``); ``load`` returns a ``TranslatedLayer`` that
runs it.
"""
from __future__ import annotations

import functools
import os

import torch

from ..framework.tensor import Tensor

_enabled = [True]


class InputSpec:
    def __init__(self, shape=None, dtype="float32", name=None, stop_gradient=False):
        self.shape = list(shape) if shape is not None else None
        self.dtype = dtype
        self.name = name
        self.stop_gradient = stop_gradient

    @classmethod
    def from_tensor(cls, tensor, name=None):
        return cls(tensor.shape, tensor.dtype, name or getattr(tensor, "name", None))

    def __repr__(self):
        return f"InputSpec(shape={self.shape}, dtype={self.dtype}, name={self.name})"


def _sig(args):
    out = []
    for a in args:
        if isinstance(a, Tensor):
            out.append(("T", tuple(a.shape), str(a.dtype), str(a._t.device)))
        else:
            out.append(("C", repr(a)))
    return tuple(out)


class StaticFunction:
    def __init__(self, fn, input_spec=None, build_strategy=None, layer=None):
        self._fn = fn
        self._layer = layer
        self._input_spec = input_spec
        self._build_strategy = build_strategy
        self._cache = {}
        functools.update_wrapper(self, fn)

    def _record(self, args):
        from .. import static
        from ..static import graph as g

        prog = static.Program()
        was = g._state.static
        g._state.static = True
        try:
            with static.program_guard(prog, static.Program()):
                sym_args, feeds = [], []
                specs = list(self._input_spec or [])
                for i, a in enumerate(args):
                    if isinstance(a, Tensor):
                        sp = specs[i] if i < len(specs) else None
                        name = getattr(sp, "name", None) or f"input_{i}"
                        v = static.data(name, list(a.shape), a.dtype)
                        sym_args.append(v)
                        feeds.append(name)
                    else:
                        sym_args.append(a)
                fn = self._converted()
                out = fn(*sym_args) if self._layer is None else fn(self._layer, *sym_args)
        finally:
            g._state.static = was
        single = isinstance(out, Tensor)
        outs = [out] if single else list(out)
        return prog, feeds, outs, single

    def _converted(self):
        """The dy2static-converted function: tensor-dependent ``if`` / ``while`` become static.nn.cond /
        while_loop while recording (jit/dy2static.py); unconvertible functions are used as written."""
        if not hasattr(self, "_conv"):
            from .dy2static import convert_function

            try:
                self._conv = convert_function(self._fn)
            except (SyntaxError, TypeError, ValueError):
                self._conv = self._fn
        return self._conv

    def get_program(self, *args):
        key = _sig(args)
        if key not in self._cache:
            self._cache[key] = self._record(args)
        return self._cache[key]

    def __call__(self, *args, **kwargs):
        if not _enabled[0] or kwargs:
            return self._fn(*args, **kwargs) if self._layer is None else self._fn(self._layer, *args, **kwargs)
        from ..static import CompiledProgram, Executor

        prog, feeds, outs, single = self.get_program(*args)
        exe = Executor(args[0]._t.device if args and isinstance(args[0], Tensor) else None)
        target = CompiledProgram(prog, self._build_strategy) if self._build_strategy is not None else prog
        feed = {n: a for n, a in zip(feeds, [a for a in args if isinstance(a, Tensor)])}
        res = exe.run(target, feed=feed, fetch_list=outs, return_numpy=False, _grad=torch.is_grad_enabled())
        return res[0] if single else tuple(res)

    def __get__(self, obj, objtype=None):
        """``@to_static`` on a method: bind the instance; the bound StaticFunction (and its per-signature
        Program cache) lives on the instance so repeated calls replay instead of re-recording."""
        if obj is None or self._layer is not None:
            return self
        key = f"_pd_static_{id(self)}"
        bound = obj.__dict__.get(key)
        if bound is None:
            bound = StaticFunction(self._fn, self._input_spec, self._build_strategy, layer=obj)
            obj.__dict__[key] = bound
        return bound

    @property
    def concrete_program(self):
        if not self._cache:
            return None
        return next(iter(self._cache.values()))[0]


def to_static(function=None, input_spec=None, build_strategy=None, backend=None, full_graph=None, **kwargs):
    """full_graph=True: AST mode (dy2static conversion, one Program per input signature; an unconvertible
    construct raises).  full_graph=False: SOT mode (jit/sot.py — guarded Program cache, graph breaks fall back to
    dygraph at Layer granularity).  Unset: ENABLE_FALL_BACK (reference jit/api.py:109) picks; this framework's
    default is AST mode, whose conversion already captures tensor-dependent control flow."""
    if full_graph is None:
        from .sot import enabled_by_env

        full_graph = not enabled_by_env()

    def deco(fn):
        from ..nn.layer.layers import Layer

        if not full_graph:
            from .sot import SymbolicTranslator, _BoundForward

            if isinstance(fn, Layer):
                fn._dygraph_forward = fn.forward
                fn._input_spec = input_spec
                fn.forward = _BoundForward(SymbolicTranslator(type(fn).forward, layer=fn,
                                                              build_strategy=build_strategy))
                return fn
            return SymbolicTranslator(fn, build_strategy=build_strategy)
        if isinstance(fn, Layer):
            sf = StaticFunction(type(fn).forward, input_spec, build_strategy, layer=fn)
            fn._static_forward = sf
            fn._input_spec = input_spec
            orig_call = fn.forward

            def fwd(*a, **k):
                return sf(*a, **k)

            fn.forward = fwd
            fn._dygraph_forward = orig_call
            return fn
        return StaticFunction(fn, input_spec, build_strategy)

    return deco(function) if function is not None else deco


def not_to_static(fn):
    return fn


def ignore_module(modules):
    pass


def enable_to_static(enable):
    _enabled[0] = bool(enable)


def _spec_tensors(input_spec):
    out = []
    for s in input_spec:
        if isinstance(s, Tensor):
            out.append(s)
        else:
            shp = [1 if (d is None or d < 0) else d for d in s.shape]
            from ..framework.dtype import convert_dtype

            dt = convert_dtype(s.dtype)
            out.append(Tensor._wrap(torch.zeros(shp, dtype=dt)))
    return out


def save(layer, path, input_spec=None, **configs):
    """Record the layer's inference Program for ``input_spec`` and write .pdmodel / .pdiparams."""
    from .. import static

    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    spec = input_spec or getattr(layer, "_input_spec", None)
    assert spec, "jit.save needs input_spec (or a to_static layer with one)"
    was_training = getattr(layer, "training", False)
    if hasattr(layer, "eval"):
        layer.eval()
    fwd = getattr(layer, "_dygraph_forward", None) or layer.forward
    sf = StaticFunction(lambda *a: fwd(*a), spec)
    prog, feeds, outs, single = sf._record(_spec_tensors(spec))
    with torch.no_grad():
        static.save_inference_model(path, [Tensor._wrap(prog.feeds[n]) for n in feeds], outs, program=prog)
    if was_training and hasattr(layer, "train"):
        layer.train()


class TranslatedLayer:
    """A loaded inference Program callable like a Layer."""

    def __init__(self, program, feeds, fetch):
        from ..static import Executor

        self._program, self._feeds, self._fetch = program, feeds, fetch
        self._exe = Executor()
        self.training = False

    def __call__(self, *args):
        feed = dict(zip(self._feeds, args))
        res = self._exe.run(self._program, feed=feed, fetch_list=self._fetch, return_numpy=False)
        return res[0] if len(res) == 1 else tuple(res)

    forward = __call__

    def eval(self):
        return self

    def train(self):
        return self

    def program(self):
        return self._program

    def state_dict(self):
        return {}


def load(path, **configs):
    from ..static import load_inference_model

    prog, feeds, fetch = load_inference_model(path)
    return TranslatedLayer(prog, feeds, fetch)
