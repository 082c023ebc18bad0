"""SOT-mode to_static: guarded program cache with graph-break fallback (reference python/paddle/jit/sot/ —
``symbolic_translate`` / ``SymbolicStaticFunction``, dy2static/program_translator.py:752).

The reference translates CPython bytecode (an eval-frame hook simulates every opcode, builds a FunctionGraph,
guards the result and, on an unsupported construct, compiles the graph so far and resumes the rest eagerly).  This
framework gets the same user-visible contract without a bytecode interpreter:

* **guards** — a translated call is keyed by a guard over everything the recorded Program baked in: tensor
  metadata (shape, dtype, device, stop_gradient), Python scalar / string argument VALUES, the bound layer's
  ``training`` flag and the scalar globals the function's code reads (``co_names`` resolved in
  ``__globals__``).  A guard miss records a new Program (dy2static AST conversion first, so tensor ``if`` /
  ``while`` / early ``return`` / ``break`` are captured); a guard hit replays the cached Program through the
  Executor (hipGraph replay under ``build_strategy.enable_cuda_graph``);
* **graph breaks** — when recording needs a concrete value (``bool`` / ``item`` / ``numpy`` of a symbolic
  tensor, an unconvertible construct), that guard key is marked eager and the call runs in dygraph.  For a
  Layer, the break is then pushed DOWN one level: every direct sub-layer gets its own translator, so the
  sub-layers that do trace run as compiled Programs while only the breaking code stays eager — the
  Layer-granularity analogue of SOT's "compile the prefix, fall back, resume";
* **stats** — per-function counters (programs compiled, guard hits, graph breaks with reasons, eager calls)
  through ``translator.stats`` and ``sot.summary()`` (reference sot/utils GraphLogger / StepInfoManager).
"""
from __future__ import annotations

import functools
import inspect
import os
import types
import weakref

from ..framework.tensor import Tensor

_SCALARS = (bool, int, float, str, type(None))
_all_translators = weakref.WeakSet()


def enabled_by_env():
    """ENABLE_FALL_BACK (reference jit/api.py:109): to_static's default mode when full_graph is not given."""
    return os.environ.get("ENABLE_FALL_BACK", "0").lower() in ("1", "true", "on")


class GraphBreak(Exception):
    pass


def _is_sym(t):
    from ..static.nn import _is_sym as s

    return s(t)


def _arg_guard(a, depth=0):
    if isinstance(a, Tensor):
        return ("T", tuple(a.shape), str(a.dtype), str(a._t.device), bool(a.stop_gradient))
    if isinstance(a, _SCALARS):
        return ("V", type(a).__name__, a)
    if isinstance(a, (list, tuple)) and depth < 4:
        return (type(a).__name__,) + tuple(_arg_guard(x, depth + 1) for x in a)
    if isinstance(a, dict) and depth < 4:
        return ("dict",) + tuple((k, _arg_guard(v, depth + 1)) for k, v in sorted(a.items(), key=lambda kv: str(kv[0])))
    training = getattr(a, "training", None)
    return ("O", type(a).__qualname__, id(a), training)


def _global_guard(fn):
    code = getattr(fn, "__code__", None)
    glb = getattr(fn, "__globals__", {})
    if code is None:
        return ()
    out = []
    for name in code.co_names:
        if name in glb and isinstance(glb[name], _SCALARS):
            out.append((name, glb[name]))
    return tuple(out)


def _is_static_capable(args):
    """The Program path takes tensors and constants positionally (StaticFunction contract)."""
    return all(isinstance(a, Tensor) or isinstance(a, _SCALARS) for a in args)


class SymbolicTranslator:
    """One translated function (optionally bound to a Layer)."""

    def __init__(self, fn, layer=None, build_strategy=None, training=None):
        self._fn = fn
        self._layer = layer
        self._build_strategy = build_strategy
        self._training = training
        self._programs = {}      # guard -> StaticFunction holding that guard's Program (Program-level mode)
        self._traces = {}        # guard -> [opcode_executor.Trace] (bytecode mode)
        self._eager = {}         # guard -> break reason
        self._children_done = False
        self.stats = {"compiled": 0, "guard_hits": 0, "graph_breaks": 0, "eager_calls": 0, "breaks": [],
                      "simulations": 0, "trace_misses": 0}
        try:
            self._sig = inspect.signature(fn)
        except (TypeError, ValueError):
            self._sig = None
        functools.update_wrapper(self, fn)
        _all_translators.add(self)

    # ------------------------------------------------------------------ helpers
    def _positional(self, args, kwargs):
        if not kwargs or self._sig is None:
            return args, kwargs
        full = ((self._layer,) + tuple(args)) if self._layer is not None else tuple(args)
        try:
            ba = self._sig.bind(*full, **kwargs)
        except TypeError:
            return args, kwargs
        ba.apply_defaults()
        if any(p.kind in (p.VAR_POSITIONAL, p.VAR_KEYWORD) for p in self._sig.parameters.values()):
            return args, kwargs
        pos = tuple(ba.arguments.values())
        return (pos[1:] if self._layer is not None else pos), {}

    def _guard(self, args):
        layer_state = (getattr(self._layer, "training", None),) if self._layer is not None else ()
        return (tuple(_arg_guard(a) for a in args), _global_guard(self._fn), layer_state)

    def _run_eager(self, args, kwargs):
        self.stats["eager_calls"] += 1
        if self._layer is not None and not self._children_done:
            self._translate_children()
        return self._fn(*args, **kwargs) if self._layer is None else self._fn(self._layer, *args, **kwargs)

    def _translate_children(self):
        """Graph break inside a Layer: give every direct sub-layer its own translator."""
        from ..nn.layer.layers import Layer

        self._children_done = True
        for child in self._layer.children():
            if not isinstance(child, Layer) or isinstance(child.__dict__.get("forward"), _BoundForward):
                continue
            child.forward = _BoundForward(SymbolicTranslator(type(child).forward, layer=child,
                                                             build_strategy=self._build_strategy))

    # ------------------------------------------------------------------ call
    def __call__(self, *args, **kwargs):
        from . import StaticFunction

        from ..static import graph as g

        if g._state.static or any(isinstance(a, Tensor) and _is_sym(a) for a in args):
            # called while an enclosing translator records: inline into that Program
            return self._fn(*args, **kwargs) if self._layer is None else self._fn(self._layer, *args, **kwargs)
        args, kwargs = self._positional(args, kwargs)
        from . import opcode_executor as oe

        if oe.enabled() and not kwargs:
            return self._call_bytecode(args)
        if kwargs or not _is_static_capable(args):
            return self._run_eager(args, kwargs)
        key = self._guard(args)
        if key in self._eager:
            return self._run_eager(args, kwargs)
        sf = self._programs.get(key)
        if sf is None:
            sf = StaticFunction(self._fn, None, self._build_strategy, layer=self._layer)
            try:
                sf.get_program(*args)
            except Exception as e:  # noqa: BLE001 — any failure to record is a graph break for this guard
                reason = f"{type(e).__name__}: {e}"[:300]
                self._eager[key] = reason
                self.stats["graph_breaks"] += 1
                self.stats["breaks"].append(reason)
                return self._run_eager(args, kwargs)
            self._programs[key] = sf
            self.stats["compiled"] += 1
        else:
            self.stats["guard_hits"] += 1
        return sf(*args)

    # ------------------------------------------------------------------ bytecode mode (jit/opcode_executor.py)
    MAX_TRACES = 8

    def _call_bytecode(self, args):
        """Replay a recorded trace of this guard if one applies; otherwise simulate the bytecode (sub-graphs split
        at the graph breaks) and keep the new trace."""
        from . import opcode_executor as oe

        key = self._guard(args)
        if key in self._eager:
            return self._run_eager(args, {})
        full = ((self._layer,) + tuple(args)) if self._layer is not None else tuple(args)
        for tr in self._traces.get(key, ()):
            try:
                out = oe.replay(tr, full)
            except oe.TraceMiss:
                self.stats["trace_misses"] += 1
                continue
            self.stats["guard_hits"] += 1
            return out
        try:
            res, tr = oe.translate_call(self._fn, full, None, self._build_strategy)
        except oe.Unsupported as e:
            reason = f"Unsupported: {e}"[:300]
            self._eager[key] = reason
            self.stats["breaks"].append(reason)
            return self._run_eager(args, {})
        self.stats["simulations"] += 1
        self.stats["compiled"] += tr.n_graphs
        self.stats["graph_breaks"] += tr.n_breaks
        if tr.n_breaks:
            self.stats["breaks"].append(f"{tr.n_breaks} break(s) in {self._fn.__qualname__}")
        if tr.replayable:
            lst = self._traces.setdefault(key, [])
            if len(lst) < self.MAX_TRACES:
                lst.append(tr)
        return res

    @property
    def traces(self):
        return [t for ts in self._traces.values() for t in ts]

    def __get__(self, obj, objtype=None):
        if obj is None or self._layer is not None:
            return self
        key = f"_pd_sot_{id(self)}"
        bound = obj.__dict__.get(key)
        if bound is None:
            bound = SymbolicTranslator(self._fn, layer=obj, build_strategy=self._build_strategy)
            obj.__dict__[key] = bound
        return bound

    @property
    def concrete_programs(self):
        return [sf.concrete_program for sf in self._programs.values()]


class _BoundForward:
    """``layer.forward`` replacement calling its translator (keeps Layer.__call__ hooks intact)."""

    def __init__(self, tr):
        self.translator = tr

    def __call__(self, *a, **k):
        return self.translator(*a, **k)


def symbolic_translate(fn, build_strategy=None, training=True, backend=None, **kwargs):
    """Reference sot/translate.py symbolic_translate: a guarded, graph-breaking translation of ``fn``."""
    if isinstance(fn, types.MethodType):
        return SymbolicTranslator(fn.__func__, layer=fn.__self__, build_strategy=build_strategy, training=training)
    return SymbolicTranslator(fn, build_strategy=build_strategy, training=training)


def summary():
    """Aggregate counters over every live translator (reference sot GraphLogger.print_info)."""
    out = {"translators": 0, "compiled": 0, "guard_hits": 0, "graph_breaks": 0, "eager_calls": 0}
    for t in list(_all_translators):
        out["translators"] += 1
        for k in ("compiled", "guard_hits", "graph_breaks", "eager_calls"):
            out[k] += t.stats[k]
    return out
