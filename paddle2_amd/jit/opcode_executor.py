"""Bytecode-level symbolic translation for SOT mode (reference python/paddle/jit/sot/: opcode_translator/executor/
opcode_executor.py simulates CPython opcodes into a FunctionGraph, guards the result and, at an unsupported
construct, compiles the graph so far, runs the construct eagerly and carries on).

CPython 3.10 bytecode is SIMULATED instruction by instruction (``OpcodeExecutor``) over a private value stack,
locals and cells, with every tensor of the frame turned into a symbolic Variable of the current sub-graph (a static
``Program``).  Tensor operations on them record into that Program; everything else (Python scalars, containers,
attribute loads, calls of library code) executes concretely.  A graph break happens MID-FUNCTION when

* a conditional jump tests a symbolic tensor (``if x.sum() > 0:``), or
* a call needs a concrete value (``int(t)``, ``t.numpy()``, ``print(t.item())``, an op that refuses symbolic input):

the current sub-graph is closed (its live tensors — every symbolic value in the stack, the locals and the cells of
all simulated frames — are fetched by running it through the Executor), the jump / call runs on the concrete
values, and a new sub-graph starts from the instruction after it.  Calls of plain user Python functions (and the
``forward`` of hook-free user Layers) are simulated inline in a child frame, so a break inside them is a break at
that instruction too.  A ``with`` block breaks the graph at its ``__enter__`` and at its ``__exit__`` (both run
concretely and are recorded as calls, so the sub-graph of the body runs INSIDE the context: ``with paddle.no_grad():``
records and replays a no-grad segment); a manager the replay cannot re-enter (a ``contextlib`` generator, one whose
constructor already changed state) makes the trace simulation-only.  Opcodes outside the supported set (``try``,
``async with``, generators) abandon the translation for the whole call (``Unsupported``: the caller runs it eagerly);
an abandoned translation leaves the contexts it entered first.

The simulation also records a ``Trace`` — the flat sequence of sub-graphs, branch outcomes, eager calls and the
return spec, over *slots* (every tensor that enters the frame: arguments, sub-graph outputs, eager-call results).
A later call whose guard matches REPLAYS the trace without simulating bytecode: sub-graphs run from the cache,
branch outcomes and the non-tensor results of eager calls are checked against what was recorded (a mismatch falls
back to a fresh simulation, which records another trace for the same guard).
"""
from __future__ import annotations

import builtins
import dis
import operator
import os
import types

import torch

from ..framework.tensor import Tensor

__all__ = ["OpcodeExecutor", "Trace", "Unsupported", "TraceMiss", "translate_call", "replay"]


class Unsupported(Exception):
    """The function uses a construct the simulator does not handle: run the whole call eagerly."""


class TraceMiss(Exception):
    """A recorded trace does not apply to this call (a branch or a guarded value differs)."""


def _is_sym_tensor(v):
    from ..static.graph import SymTensor

    return isinstance(v, Tensor) and isinstance(v._t, SymTensor)


def _is_param(v):
    return bool(getattr(v, "persistable", False)) or type(v).__name__ in ("Parameter", "EagerParamBase")


# ------------------------------------------------------------------------------------------- trace
class Trace:
    """Replayable record of one simulated call (see module doc)."""

    def __init__(self):
        self.arg_slots = []    # spec of the flattened positional arguments
        self.steps = []
        self.replayable = True
        self.n_graphs = 0
        self.n_breaks = 0

    def __repr__(self):
        kinds = [s[0] for s in self.steps]
        return f"Trace(graphs={self.n_graphs}, breaks={self.n_breaks}, steps={kinds})"


_LIB_PREFIXES = None


def _library_module(mod):
    """Code of the framework / torch / numpy / the standard library is called, not simulated."""
    global _LIB_PREFIXES
    if _LIB_PREFIXES is None:
        _LIB_PREFIXES = ("paddle2_amd", "torch", "numpy", "builtins", "functools", "typing", "collections", "math",
                         "operator", "itertools", "abc", "inspect", "copy", "contextlib", "warnings", "enum")
    if mod is None:
        return True
    return str(mod).split(".")[0] in _LIB_PREFIXES


_BINARY = {
    "BINARY_ADD": operator.add, "BINARY_SUBTRACT": operator.sub, "BINARY_MULTIPLY": operator.mul,
    "BINARY_TRUE_DIVIDE": operator.truediv, "BINARY_FLOOR_DIVIDE": operator.floordiv, "BINARY_MODULO": operator.mod,
    "BINARY_POWER": operator.pow, "BINARY_MATRIX_MULTIPLY": operator.matmul, "BINARY_SUBSCR": operator.getitem,
    "BINARY_AND": operator.and_, "BINARY_OR": operator.or_, "BINARY_XOR": operator.xor,
    "BINARY_LSHIFT": operator.lshift, "BINARY_RSHIFT": operator.rshift,
    "INPLACE_ADD": operator.iadd, "INPLACE_SUBTRACT": operator.isub, "INPLACE_MULTIPLY": operator.imul,
    "INPLACE_TRUE_DIVIDE": operator.itruediv, "INPLACE_FLOOR_DIVIDE": operator.ifloordiv,
    "INPLACE_MODULO": operator.imod, "INPLACE_POWER": operator.ipow, "INPLACE_MATRIX_MULTIPLY": operator.imatmul,
    "INPLACE_AND": operator.iand, "INPLACE_OR": operator.ior, "INPLACE_XOR": operator.ixor,
    "INPLACE_LSHIFT": operator.ilshift, "INPLACE_RSHIFT": operator.irshift,
}
_UNARY = {"UNARY_POSITIVE": operator.pos, "UNARY_NEGATIVE": operator.neg, "UNARY_NOT": operator.not_,
          "UNARY_INVERT": operator.invert}
_COMPARE = {"<": operator.lt, "<=": operator.le, "==": operator.eq, "!=": operator.ne, ">": operator.gt,
            ">=": operator.ge}


class _Method:
    """LOAD_METHOD result placeholder: the attribute is looked up on the (possibly materialised) owner at call
    time, so a break between LOAD_METHOD and CALL_METHOD sees the concrete tensor."""

    __slots__ = ("name",)

    def __init__(self, name):
        self.name = name


_NULL = object()


class _Frame:
    def __init__(self, fn, args, kwargs):
        code = fn.__code__
        if code.co_flags & (0x20 | 0x80 | 0x100 | 0x200):  # generator / coroutine / async generator
            raise Unsupported("generator or coroutine function")
        self.fn = fn
        self.code = code
        self.instrs = list(dis.get_instructions(code))
        self.index = {ins.offset: i for i, ins in enumerate(self.instrs)}
        self.glb = fn.__globals__
        self.locals = {}
        self.stack = []
        self.ip = 0
        import inspect

        ba = inspect.signature(fn).bind(*args, **kwargs)
        ba.apply_defaults()
        for k, v in ba.arguments.items():
            if k not in code.co_varnames and k.startswith("implicit") and "." + k[8:] in code.co_varnames:
                k = "." + k[8:]   # a comprehension's hidden iterator argument (inspect names ".0" "implicit0")
            self.locals[k] = v
        # cells are real cell objects: the enclosing function's cells for free variables (writes are seen outside,
        # as in CPython), fresh ones for this frame's cell variables (closures made by MAKE_FUNCTION share them)
        self.cells = {}
        for name, cell in zip(code.co_freevars, fn.__closure__ or ()):
            self.cells[name] = cell
        for name in code.co_cellvars:
            self.cells[name] = types.CellType(self.locals[name]) if name in self.locals else types.CellType()

    def jump(self, target_offset):
        self.ip = self.index[target_offset]


class OpcodeExecutor:
    """Simulate one call of ``fn`` (see module doc).  ``run()`` returns the call's result; ``self.trace`` holds the
    replayable record."""

    MAX_INSTR = 2_000_000

    def __init__(self, fn, args, kwargs=None, build_strategy=None):
        self.fn = fn
        self.args = args
        self.kwargs = kwargs or {}
        self.build_strategy = build_strategy
        self.trace = Trace()
        self.frames = []
        self.slot_of = {}      # id(Tensor) -> slot
        self.slot_val = {}     # slot -> Tensor (keeps it alive: ids stay unique)
        self.graph = None      # current sub-graph state
        self._steps = 0
        self._exits = []       # bound __exit__ of the ``with`` blocks entered and not yet left (innermost last)

    # ----------------------------------------------------------------------------------- slots & specs
    def _new_slot(self, t):
        k = len(self.slot_val)
        self.slot_val[k] = t
        self.slot_of[id(t)] = k
        return k

    def _spec(self, v, depth=0):
        """How to rebuild ``v`` at replay: tensors by slot, containers recursively, anything else by reference."""
        if isinstance(v, Tensor):
            k = self.slot_of.get(id(v))
            return ("slot", k) if k is not None else ("const", v)
        if isinstance(v, (list, tuple)) and depth < 8:
            return (type(v).__name__, tuple(self._spec(x, depth + 1) for x in v))
        if isinstance(v, dict) and depth < 8:
            return ("dict", tuple((k, self._spec(x, depth + 1)) for k, x in v.items()))
        return ("const", v)

    def _bind(self, v, depth=0):
        """Give every tensor of an eager result a slot; non-tensor leaves become guards (equality at replay)."""
        if isinstance(v, Tensor):
            return ("slot", self._new_slot(v))
        if isinstance(v, (list, tuple)) and depth < 8:
            return (type(v).__name__, tuple(self._bind(x, depth + 1) for x in v))
        if isinstance(v, dict) and depth < 8:
            return ("dict", tuple((k, self._bind(x, depth + 1)) for k, x in v.items()))
        if isinstance(v, (bool, int, float, str, bytes, type(None), complex)):
            return ("guard", v)
        self.trace.replayable = False   # an opaque object flows on: never replay, always simulate
        return ("const", v)

    # ----------------------------------------------------------------------------------- frame state
    def _map_state(self, f):
        """Apply ``f`` to every leaf of every simulated frame (stack, locals, cells), rebuilding containers."""

        def walk(v, depth=0):
            if isinstance(v, Tensor):
                return f(v)
            if isinstance(v, tuple) and depth < 8 and not hasattr(v, "_fields"):
                n = tuple(walk(x, depth + 1) for x in v)
                return n if any(a is not b for a, b in zip(n, v)) else v
            if isinstance(v, list) and depth < 8:
                n = [walk(x, depth + 1) for x in v]
                if any(a is not b for a, b in zip(n, v)):
                    v[:] = n   # in place: aliases of the list (a list being built up) stay aliases
                return v
            if isinstance(v, dict) and depth < 8:
                for k in list(v.keys()):
                    x = v[k]
                    y = walk(x, depth + 1)
                    if y is not x:
                        v[k] = y
                return v
            return v

        for fr in self.frames:
            fr.stack[:] = [walk(v) for v in fr.stack]
            for k in list(fr.locals):
                fr.locals[k] = walk(fr.locals[k])
            for c in fr.cells.values():
                try:
                    v = c.cell_contents
                except ValueError:   # empty cell
                    continue
                w = walk(v)
                if w is not v:
                    c.cell_contents = w

    def _start_graph(self):
        from .. import static
        from ..static import graph as g

        prog = static.Program()
        lifted = {}   # slot -> symbolic Tensor
        feeds = []    # (feed name, slot)

        def lift(t):
            if _is_sym_tensor(t) or _is_param(t):
                return t
            k = self.slot_of.get(id(t))
            if k is None:
                return t   # not a frame input (a buffer / constant): captured by reference
            s = lifted.get(k)
            if s is None:
                was = g._state.static
                g._state.static = True
                g._stack.append((prog, static.Program()))
                try:
                    s = static.data(f"slot{k}", list(t.shape), t.dtype)
                    s.stop_gradient = t.stop_gradient
                finally:
                    g._stack.pop()
                    g._state.static = was
                lifted[k] = s
                feeds.append((f"slot{k}", k))
            return s

        self._map_state(lift)
        self.graph = {"prog": prog, "feeds": feeds, "lifted": lifted, "was": g._state.static}
        g._state.static = True
        g._stack.append((prog, static.Program()))

    def _suspend(self):
        from ..static import graph as g

        if self.graph is not None:
            g._stack.pop()
            g._state.static = self.graph["was"]

    def _end_graph(self):
        """Close the current sub-graph: run it and replace every live symbolic tensor by its value."""
        if self.graph is None:
            return
        from ..static import Executor

        gs = self.graph
        self._suspend()
        self.graph = None
        outs, seen = [], {}
        # a lifted input still live unchanged maps back to its slot's tensor (fetching it would detach it when the
        # sub-graph runs under no_grad, and copies it for nothing otherwise)
        fed = {id(s): self.slot_val[k] for k, s in gs["lifted"].items()}

        def collect(t):
            if _is_sym_tensor(t) and id(t) not in seen and id(t) not in fed:
                seen[id(t)] = len(outs)
                outs.append(t)
            return t

        self._map_state(collect)
        if fed:
            self._map_state(lambda t: fed.get(id(t), t))
        if not outs:
            return
        prog = gs["prog"]
        exe = Executor(None)
        feed = {name: self.slot_val[k] for name, k in gs["feeds"]}
        from ..static import CompiledProgram

        target = CompiledProgram(prog, self.build_strategy) if self.build_strategy is not None else prog
        vals = exe.run(target, feed=feed, fetch_list=outs, return_numpy=False, _grad=torch.is_grad_enabled())
        vals = [v if isinstance(v, Tensor) else Tensor._wrap(v) for v in vals]
        out_slots = [self._new_slot(v) for v in vals]
        self.trace.steps.append(("graph", target, tuple(gs["feeds"]), tuple(outs), tuple(out_slots)))
        self.trace.n_graphs += 1
        by_id = {id(s): vals[i] for s, i in ((s, seen[id(s)]) for s in outs)}
        self._map_state(lambda t: by_id.get(id(t), t))

    # ----------------------------------------------------------------------------------- entry
    def run(self):
        fr = _Frame(self.fn, self.args, self.kwargs)
        # arguments enter as slots (the replay binds the same positions)
        flat = []

        def take(v, depth=0):
            if isinstance(v, Tensor):
                flat.append(self._new_slot(v))
            elif isinstance(v, (list, tuple)) and depth < 8:
                for x in v:
                    take(x, depth + 1)

        for a in self.args:
            take(a)
        self.trace.arg_slots = flat
        self.frames.append(fr)
        self._start_graph()
        try:
            ret = self._execute(fr)
        except BaseException as e:
            self._suspend()
            self.graph = None
            while self._exits:   # leave the contexts the simulation entered before the call is re-run eagerly
                self._exits.pop()(type(e), e, e.__traceback__)
            raise
        return ret

    def _execute(self, fr):
        """Run frame ``fr`` to its RETURN_VALUE; returns the value (the caller frame continues afterwards)."""
        while True:
            self._steps += 1
            if self._steps > self.MAX_INSTR:
                raise Unsupported("instruction budget exceeded")
            ins = fr.instrs[fr.ip]
            fr.ip += 1
            op = ins.opname
            if op == "RETURN_VALUE":
                v = fr.stack.pop()
                if len(self.frames) == 1:   # the translated function returns: close the graph
                    fr.stack.append(v)
                    self._end_graph()
                    v = fr.stack.pop()
                    self.trace.steps.append(("return", self._spec(v)))
                return v
            h = getattr(self, "op_" + op, None)
            if h is not None:
                h(fr, ins)
            elif op in _BINARY:
                b = fr.stack.pop()
                a = fr.stack.pop()
                fr.stack.append(self._apply(_BINARY[op], (a, b)))
            elif op in _UNARY:
                if op == "UNARY_NOT" and _is_sym_tensor(fr.stack[-1]):
                    self._break_on_top(fr)
                fr.stack.append(self._apply(_UNARY[op], (fr.stack.pop(),)))
            else:
                raise Unsupported(f"opcode {op}")

    # ----------------------------------------------------------------------------------- calls / breaks
    def _apply(self, f, args, kwargs=None):
        """Call ``f`` on frame values: symbolically when possible; a failure with symbolic operands is a graph
        break — the sub-graph is closed, the call runs on concrete values and a new sub-graph starts."""
        kwargs = kwargs or {}
        sym = any(_is_sym_tensor(a) for a in args) or any(_is_sym_tensor(v) for v in kwargs.values()) or (
            isinstance(f, types.MethodType) and _is_sym_tensor(f.__self__))
        prog = self.graph["prog"] if self.graph is not None else None
        n0 = len(prog.ops) if prog is not None else 0
        try:
            return f(*args, **kwargs)
        except (Unsupported, TraceMiss):
            raise
        except Exception:   # noqa: BLE001
            if not sym and not any(_is_sym_tensor(x) for x in self._flat_leaves((args, kwargs))):
                raise
            if prog is not None:
                del prog.ops[n0:]   # drop whatever the failed attempt recorded
        return self._eager_call(f, args, kwargs)

    @staticmethod
    def _flat_leaves(v, depth=0):
        if isinstance(v, (list, tuple)) and depth < 8:
            for x in v:
                yield from OpcodeExecutor._flat_leaves(x, depth + 1)
        elif isinstance(v, dict) and depth < 8:
            for x in v.values():
                yield from OpcodeExecutor._flat_leaves(x, depth + 1)
        else:
            yield v

    def _eager_call(self, f, args, kwargs):
        """Graph break at a call: materialise, call concretely, record the call for replay."""
        fr = self.frames[-1]
        # put the call's operands on the stack so materialisation replaces them, then take them back
        owner = f.__self__ if isinstance(f, types.MethodType) and isinstance(f.__self__, Tensor) else None
        fr.stack.append([owner, list(args), dict(kwargs)])
        self._end_graph()
        owner, args, kwargs = fr.stack.pop()
        if owner is not None:
            f = getattr(owner, f.__name__)
            fspec = ("method", self._spec(owner), f.__name__)
        else:
            fspec = ("const", f)
        aspec = self._spec(list(args))
        kspec = self._spec(dict(kwargs))
        r = f(*args, **kwargs)
        rspec = self._bind(r)
        self.trace.steps.append(("call", fspec, aspec, kspec, rspec))
        self.trace.n_breaks += 1
        self._start_graph()
        return r

    def _ctx_call(self, f, args, mgr):
        """Graph break at a context manager's ``__enter__`` / ``__exit__``: the sub-graph so far runs before it (a
        body's graph runs inside the context), the call runs concretely and is recorded for replay."""
        fr = self.frames[-1]
        fr.stack.append(list(args))
        self._end_graph()
        args = fr.stack.pop()
        aspec = self._spec(list(args))
        r = f(*args)
        rspec = ("const", r) if r is mgr or r is None else self._bind(r)
        self.trace.steps.append(("call", ("const", f), aspec, ("dict", ()), rspec))
        self.trace.n_breaks += 1
        self._start_graph()
        return r

    def _break_on_top(self, fr):
        """TOS is a symbolic tensor a jump / ``not`` tests: materialise it and record the branch outcome."""
        self._end_graph()
        v = fr.stack[-1]
        b = bool(v)
        self.trace.steps.append(("branch", self._spec(v), b))
        self.trace.n_breaks += 1
        self._start_graph()
        return b

    def _truth(self, fr):
        v = fr.stack[-1]
        if _is_sym_tensor(v):
            return self._break_on_top(fr)
        return bool(v)

    def _call(self, fr, f, args, kwargs):
        # user Python functions (and hook-free user Layers' forward) are simulated inline: a break inside them is
        # a break at that instruction, not at the call
        target = None
        if isinstance(f, types.FunctionType) and not _library_module(getattr(f, "__module__", None)):
            target, targs = f, list(args)
        elif isinstance(f, types.MethodType) and isinstance(f.__func__, types.FunctionType) and not _library_module(
                getattr(f.__func__, "__module__", None)):
            target, targs = f.__func__, [f.__self__] + list(args)
        else:
            from ..nn.layer.layers import Layer

            if isinstance(f, Layer) and not _library_module(type(f).__module__) and not self._has_hooks(f):
                fwd = type(f).forward
                if isinstance(fwd, types.FunctionType) and "forward" not in f.__dict__:
                    target, targs = fwd, [f] + list(args)
        if target is not None and not (target.__code__.co_flags & (0x20 | 0x80 | 0x100 | 0x200)):
            child = _Frame(target, targs, kwargs)
            self.frames.append(child)
            try:
                return self._execute(child)
            finally:
                self.frames.pop()
        return self._apply(f, args, kwargs)

    @staticmethod
    def _has_hooks(layer):
        for name in ("_forward_pre_hooks", "_forward_post_hooks"):
            if getattr(layer, name, None):
                return True
        return False

    # ----------------------------------------------------------------------------------- opcodes
    def op_NOP(self, fr, ins):
        pass

    op_EXTENDED_ARG = op_NOP

    def op_POP_TOP(self, fr, ins):
        fr.stack.pop()

    def op_ROT_TWO(self, fr, ins):
        s = fr.stack
        s[-1], s[-2] = s[-2], s[-1]

    def op_ROT_THREE(self, fr, ins):
        s = fr.stack
        s[-1], s[-2], s[-3] = s[-2], s[-3], s[-1]

    def op_ROT_FOUR(self, fr, ins):
        s = fr.stack
        s[-1], s[-2], s[-3], s[-4] = s[-2], s[-3], s[-4], s[-1]

    def op_ROT_N(self, fr, ins):
        n = ins.arg
        s = fr.stack
        s[-n:] = [s[-1]] + s[-n:-1]

    def op_DUP_TOP(self, fr, ins):
        fr.stack.append(fr.stack[-1])

    def op_DUP_TOP_TWO(self, fr, ins):
        fr.stack.extend(fr.stack[-2:])

    def op_LOAD_CONST(self, fr, ins):
        fr.stack.append(ins.argval)

    def op_LOAD_FAST(self, fr, ins):
        if ins.argval not in fr.locals:
            raise UnboundLocalError(f"local variable '{ins.argval}' referenced before assignment")
        fr.stack.append(fr.locals[ins.argval])

    def op_STORE_FAST(self, fr, ins):
        fr.locals[ins.argval] = fr.stack.pop()

    def op_DELETE_FAST(self, fr, ins):
        del fr.locals[ins.argval]

    def op_LOAD_GLOBAL(self, fr, ins):
        name = ins.argval
        if name in fr.glb:
            fr.stack.append(fr.glb[name])
        elif hasattr(builtins, name):
            fr.stack.append(getattr(builtins, name))
        else:
            raise NameError(f"name '{name}' is not defined")

    def op_LOAD_DEREF(self, fr, ins):
        try:
            fr.stack.append(fr.cells[ins.argval].cell_contents)
        except ValueError:
            raise NameError(f"free variable '{ins.argval}' referenced before assignment") from None

    op_LOAD_CLASSDEREF = op_LOAD_DEREF

    def op_STORE_DEREF(self, fr, ins):
        fr.cells[ins.argval].cell_contents = fr.stack.pop()

    def op_DELETE_DEREF(self, fr, ins):
        del fr.cells[ins.argval].cell_contents

    def op_LOAD_CLOSURE(self, fr, ins):
        fr.stack.append(fr.cells[ins.argval])

    def op_LOAD_ATTR(self, fr, ins):
        o = fr.stack.pop()
        fr.stack.append(self._apply(getattr, (o, ins.argval)))

    def op_STORE_ATTR(self, fr, ins):
        o = fr.stack.pop()
        v = fr.stack.pop()
        setattr(o, ins.argval, v)

    def op_LOAD_METHOD(self, fr, ins):
        o = fr.stack.pop()
        fr.stack.append(_Method(ins.argval))
        fr.stack.append(o)

    def op_CALL_METHOD(self, fr, ins):
        n = ins.arg
        args = fr.stack[len(fr.stack) - n:] if n else []
        del fr.stack[len(fr.stack) - n:]
        owner = fr.stack.pop()
        m = fr.stack.pop()
        f = getattr(owner, m.name) if isinstance(m, _Method) else m
        fr.stack.append(self._call(fr, f, args, {}))

    def op_CALL_FUNCTION(self, fr, ins):
        n = ins.arg
        args = fr.stack[len(fr.stack) - n:] if n else []
        del fr.stack[len(fr.stack) - n:]
        f = fr.stack.pop()
        if self._exits and n == 3 and any(f is e for e in self._exits):   # the normal exit of a ``with`` block
            self._exits = [e for e in self._exits if e is not f]
            fr.stack.append(self._ctx_call(f, args, f.__self__))
            return
        fr.stack.append(self._call(fr, f, args, {}))

    def op_SETUP_WITH(self, fr, ins):
        mgr = fr.stack.pop()
        if isinstance(mgr, Tensor):
            raise Unsupported("with over a tensor")
        cls = type(mgr)
        enter, exit_ = cls.__enter__.__get__(mgr, cls), cls.__exit__.__get__(mgr, cls)
        if not _reusable_ctx(mgr):
            self.trace.replayable = False   # the replay would re-enter a spent / pre-applied manager
        fr.stack.append(exit_)
        self._exits.append(exit_)
        fr.stack.append(self._ctx_call(enter, (), mgr))

    def op_POP_BLOCK(self, fr, ins):
        pass   # the simulator keeps no block stack: exceptions leave the simulation (see run())

    def op_CALL_FUNCTION_KW(self, fr, ins):
        names = fr.stack.pop()
        n = ins.arg
        vals = fr.stack[len(fr.stack) - n:]
        del fr.stack[len(fr.stack) - n:]
        f = fr.stack.pop()
        npos = n - len(names)
        fr.stack.append(self._call(fr, f, vals[:npos], dict(zip(names, vals[npos:]))))

    def op_CALL_FUNCTION_EX(self, fr, ins):
        kw = fr.stack.pop() if ins.arg & 1 else {}
        args = fr.stack.pop()
        f = fr.stack.pop()
        fr.stack.append(self._call(fr, f, list(args), dict(kw)))

    def op_COMPARE_OP(self, fr, ins):
        b = fr.stack.pop()
        a = fr.stack.pop()
        fr.stack.append(self._apply(_COMPARE[ins.argval], (a, b)))

    def op_IS_OP(self, fr, ins):
        b = fr.stack.pop()
        a = fr.stack.pop()
        fr.stack.append((a is not b) if ins.arg else (a is b))

    def op_CONTAINS_OP(self, fr, ins):
        b = fr.stack.pop()
        a = fr.stack.pop()
        r = self._apply(operator.contains, (b, a))
        fr.stack.append((not r) if ins.arg else r)

    def op_BUILD_TUPLE(self, fr, ins):
        n = ins.arg
        v = tuple(fr.stack[len(fr.stack) - n:]) if n else ()
        del fr.stack[len(fr.stack) - n:]
        fr.stack.append(v)

    def op_BUILD_LIST(self, fr, ins):
        n = ins.arg
        v = list(fr.stack[len(fr.stack) - n:]) if n else []
        del fr.stack[len(fr.stack) - n:]
        fr.stack.append(v)

    def op_BUILD_SET(self, fr, ins):
        n = ins.arg
        v = set(fr.stack[len(fr.stack) - n:]) if n else set()
        del fr.stack[len(fr.stack) - n:]
        fr.stack.append(v)

    def op_BUILD_MAP(self, fr, ins):
        n = ins.arg
        items = fr.stack[len(fr.stack) - 2 * n:] if n else []
        del fr.stack[len(fr.stack) - 2 * n:]
        fr.stack.append({items[2 * i]: items[2 * i + 1] for i in range(n)})

    def op_BUILD_CONST_KEY_MAP(self, fr, ins):
        keys = fr.stack.pop()
        n = ins.arg
        vals = fr.stack[len(fr.stack) - n:]
        del fr.stack[len(fr.stack) - n:]
        fr.stack.append(dict(zip(keys, vals)))

    def op_BUILD_SLICE(self, fr, ins):
        if ins.arg == 3:
            c = fr.stack.pop()
            b = fr.stack.pop()
            a = fr.stack.pop()
            fr.stack.append(slice(a, b, c))
        else:
            b = fr.stack.pop()
            a = fr.stack.pop()
            fr.stack.append(slice(a, b))

    def op_BUILD_STRING(self, fr, ins):
        n = ins.arg
        v = "".join(fr.stack[len(fr.stack) - n:]) if n else ""
        del fr.stack[len(fr.stack) - n:]
        fr.stack.append(v)

    def op_FORMAT_VALUE(self, fr, ins):
        spec = fr.stack.pop() if (ins.arg & 0x04) else ""
        v = fr.stack.pop()
        conv = ins.arg & 0x03
        if conv == 1:
            v = str(v)
        elif conv == 2:
            v = repr(v)
        elif conv == 3:
            v = ascii(v)
        fr.stack.append(self._apply(format, (v, spec)))

    def op_LIST_APPEND(self, fr, ins):
        v = fr.stack.pop()
        fr.stack[-ins.arg].append(v)

    def op_SET_ADD(self, fr, ins):
        v = fr.stack.pop()
        fr.stack[-ins.arg].add(v)

    def op_MAP_ADD(self, fr, ins):
        v = fr.stack.pop()
        k = fr.stack.pop()
        fr.stack[-ins.arg][k] = v

    def op_LIST_EXTEND(self, fr, ins):
        v = fr.stack.pop()
        fr.stack[-ins.arg].extend(v)

    def op_SET_UPDATE(self, fr, ins):
        v = fr.stack.pop()
        fr.stack[-ins.arg].update(v)

    def op_DICT_UPDATE(self, fr, ins):
        v = fr.stack.pop()
        fr.stack[-ins.arg].update(v)

    op_DICT_MERGE = op_DICT_UPDATE

    def op_LIST_TO_TUPLE(self, fr, ins):
        fr.stack.append(tuple(fr.stack.pop()))

    def op_UNPACK_SEQUENCE(self, fr, ins):
        v = fr.stack.pop()
        items = list(self._apply(list, (v,))) if not isinstance(v, (list, tuple)) else list(v)
        if len(items) != ins.arg:
            raise ValueError(f"cannot unpack {len(items)} values into {ins.arg}")
        fr.stack.extend(reversed(items))

    def op_UNPACK_EX(self, fr, ins):
        before, after = ins.arg & 0xFF, ins.arg >> 8
        items = list(fr.stack.pop())
        mid = items[before:len(items) - after] if after else items[before:]
        out = items[:before] + [mid] + (items[len(items) - after:] if after else [])
        fr.stack.extend(reversed(out))

    def op_STORE_SUBSCR(self, fr, ins):
        k = fr.stack.pop()
        o = fr.stack.pop()
        v = fr.stack.pop()
        self._apply(operator.setitem, (o, k, v))

    def op_DELETE_SUBSCR(self, fr, ins):
        k = fr.stack.pop()
        o = fr.stack.pop()
        del o[k]

    def op_GET_ITER(self, fr, ins):
        fr.stack.append(self._apply(iter, (fr.stack.pop(),)))

    def op_FOR_ITER(self, fr, ins):
        it = fr.stack[-1]
        try:
            v = self._apply(next, (it,))
        except StopIteration:
            fr.stack.pop()
            fr.jump(ins.argval)
            return
        fr.stack.append(v)

    def op_JUMP_FORWARD(self, fr, ins):
        fr.jump(ins.argval)

    def op_JUMP_ABSOLUTE(self, fr, ins):
        fr.jump(ins.argval)

    def op_POP_JUMP_IF_FALSE(self, fr, ins):
        t = self._truth(fr)
        fr.stack.pop()
        if not t:
            fr.jump(ins.argval)

    def op_POP_JUMP_IF_TRUE(self, fr, ins):
        t = self._truth(fr)
        fr.stack.pop()
        if t:
            fr.jump(ins.argval)

    def op_JUMP_IF_FALSE_OR_POP(self, fr, ins):
        if not self._truth(fr):
            fr.jump(ins.argval)
        else:
            fr.stack.pop()

    def op_JUMP_IF_TRUE_OR_POP(self, fr, ins):
        if self._truth(fr):
            fr.jump(ins.argval)
        else:
            fr.stack.pop()

    def op_GEN_START(self, fr, ins):
        raise Unsupported("generator")

    def op_LOAD_ASSERTION_ERROR(self, fr, ins):
        fr.stack.append(AssertionError)

    def op_RAISE_VARARGS(self, fr, ins):
        # raising ends the call: let the caller run it eagerly so the exception comes from real code
        raise Unsupported("raise")

    def op_MAKE_FUNCTION(self, fr, ins):
        """Nested functions / comprehensions / lambdas: a real function object over the frame's cells (calls of it
        are simulated inline like any user function; generator expressions run natively)."""
        qualname = fr.stack.pop()
        code = fr.stack.pop()
        closure = fr.stack.pop() if ins.arg & 0x08 else None
        annotations = fr.stack.pop() if ins.arg & 0x04 else None
        kwdefaults = fr.stack.pop() if ins.arg & 0x02 else None
        defaults = fr.stack.pop() if ins.arg & 0x01 else None
        f = types.FunctionType(code, fr.glb, code.co_name, defaults, closure)
        f.__qualname__ = qualname
        if kwdefaults:
            f.__kwdefaults__ = kwdefaults
        if annotations:
            f.__annotations__ = dict(zip(annotations[::2], annotations[1::2])) if isinstance(annotations, tuple) \
                else annotations
        f.__module__ = fr.glb.get("__name__")
        fr.stack.append(f)


def _reusable_ctx(mgr):
    """Managers whose ``__enter__`` holds all their effect and that can be entered again (the replay re-runs the
    recorded ``__enter__`` / ``__exit__`` on the same object)."""
    from ..framework import grad_mode

    if getattr(mgr, "_sot_reusable", False):
        return True
    return type(mgr) in (grad_mode.no_grad, grad_mode.enable_grad, torch.no_grad, torch.enable_grad)


# ------------------------------------------------------------------------------------------- replay
def _build(spec, vals):
    kind = spec[0]
    if kind == "slot":
        return vals[spec[1]]
    if kind == "const":
        return spec[1]
    if kind in ("list", "tuple"):
        items = [_build(s, vals) for s in spec[1]]
        return items if kind == "list" else tuple(items)
    if kind == "dict":
        return {k: _build(s, vals) for k, s in spec[1]}
    if kind == "guard":
        return spec[1]
    raise ValueError(spec)


def _match(spec, v, vals):
    kind = spec[0]
    if kind == "slot":
        if not isinstance(v, Tensor):
            raise TraceMiss("eager result is no longer a tensor")
        vals[spec[1]] = v
    elif kind in ("list", "tuple"):
        if not isinstance(v, (list, tuple)) or len(v) != len(spec[1]):
            raise TraceMiss("eager result structure changed")
        for s, x in zip(spec[1], v):
            _match(s, x, vals)
    elif kind == "dict":
        if not isinstance(v, dict) or set(v) != {k for k, _ in spec[1]}:
            raise TraceMiss("eager result keys changed")
        for k, s in spec[1]:
            _match(s, v[k], vals)
    elif kind == "guard":
        if type(v) is not type(spec[1]) or v != spec[1]:
            raise TraceMiss(f"guarded value changed: {spec[1]!r} -> {v!r}")


def replay(trace, args):
    """Run a recorded trace on new arguments (same guard); raises TraceMiss if it does not apply."""
    from ..static import Executor

    vals = {}
    flat = []

    def take(v, depth=0):
        if isinstance(v, Tensor):
            flat.append(v)
        elif isinstance(v, (list, tuple)) and depth < 8:
            for x in v:
                take(x, depth + 1)

    for a in args:
        take(a)
    if len(flat) != len(trace.arg_slots):
        raise TraceMiss("argument structure changed")
    for k, t in zip(trace.arg_slots, flat):
        vals[k] = t
    exe = Executor(None)
    for st in trace.steps:
        kind = st[0]
        if kind == "graph":
            _, target, feeds, fetch, out_slots = st
            res = exe.run(target, feed={n: vals[k] for n, k in feeds}, fetch_list=list(fetch), return_numpy=False,
                          _grad=torch.is_grad_enabled())
            for k, v in zip(out_slots, res):
                vals[k] = v if isinstance(v, Tensor) else Tensor._wrap(v)
        elif kind == "branch":
            if bool(_build(st[1], vals)) != st[2]:
                raise TraceMiss("branch outcome differs")
        elif kind == "call":
            _, fspec, aspec, kspec, rspec = st
            if fspec[0] == "method":
                f = getattr(_build(fspec[1], vals), fspec[2])
            else:
                f = fspec[1]
            r = f(*_build(aspec, vals), **_build(kspec, vals))
            _match(rspec, r, vals)
        elif kind == "return":
            return _build(st[1], vals)
    raise TraceMiss("trace has no return")


def translate_call(fn, args, kwargs=None, build_strategy=None):
    """Simulate one call; returns (result, trace)."""
    ex = OpcodeExecutor(fn, args, kwargs, build_strategy)
    res = ex.run()
    return res, ex.trace


def enabled():
    """Bytecode translation is the SOT mode's engine; PADDLE2_AMD_SOT_BYTECODE=0 keeps the Program-level mode."""
    return os.environ.get("PADDLE2_AMD_SOT_BYTECODE", "1") != "0"
