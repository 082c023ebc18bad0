"""Static-graph Program capture.

Reference: the static graph stack (python/paddle/static, paddle/fluid/framework ProgramDesc /
BlockDesc / OpDesc, the new IR + PIR interpreter ``StandaloneExecutor``).  Design here: a Program
is an ordered op list recorded from ordinary paddle2_amd code run on *symbolic* tensors:

  * a ``Variable`` (``paddle.static.data`` / op results) wraps a ``SymTensor`` — a torch tensor
    subclass living on the ``meta`` device, so every op gets exact shape/dtype inference for free;
  * ``SymTensor.__torch_function__`` records each torch op touching a symbolic tensor (args with
    symbolic tensors replaced by variable ids; parameters and other real tensors kept by reference,
    so optimizer updates are seen at run time);
  * the entry points of our native HIP kernels (``paddle2_amd.ops.torch_ops``: fused norms, RoPE,
    SwiGLU, flash attention, softmax-CE, embedding, ...) are recorded as ONE op each (``graph_op``),
    so an executed Program runs the same MFMA kernels as dygraph;
  * backward / optimizer steps are recorded as ``backward`` / ``optimize`` ops that drive the
    autograd engine and the fused optimizer at run time.

The Executor (static/executor.py) replays the op list on real tensors and can capture a
static-shape Program in a HIP graph (``BuildStrategy.enable_cuda_graph``) — HIP graphs instead of
a tracing compiler.
"""
from __future__ import annotations

import contextlib
import functools
import itertools

import torch
from torch.utils import _pytree as pytree

_ids = itertools.count(1)


class _State:
    static = False          # paddle.enable_static()
    recording_off = 0       # >0 while computing meta shapes inside a recorded op
    op_device = None        # static.device_guard: "gpu:<stage>" / "gpu:all" stamped on recorded ops


_state = _State()


def in_static_mode():
    return _state.static


class SymTensor(torch.Tensor):
    """Symbolic value of a static Program (meta-device storage + a variable id)."""

    @staticmethod
    def __new__(cls, meta, program, vid=None, name=None):
        r = torch.Tensor._make_subclass(cls, meta, False)
        r._program = program
        r._vid = vid if vid is not None else next(_ids)
        r._name = name
        return r

    def __repr__(self):
        return f"SymTensor(id={self._vid}, shape={tuple(self.shape)}, dtype={self.dtype})"

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if _state.recording_off:
            with torch._C.DisableTorchFunctionSubclass():
                return func(*args, **kwargs)
        prog = _find_program((args, kwargs))
        return prog._record(func, args, kwargs, kind="torch")

    @property
    def device(self):
        """The device the Program will RUN on (storage is meta only for shape inference), so code
        that builds constants "on x.device" (RoPE tables, aranges, masks) builds real ones."""
        from ..framework.place import current_torch_device

        return current_torch_device()

    @property
    def is_cuda(self):
        return self.device.type == "cuda"

    # data-dependent conversions cannot be answered at build time
    def item(self):
        raise RuntimeError("a static-graph Variable has no value at build time (use Executor.run)")

    def tolist(self):
        self.item()

    def __bool__(self):
        self.item()

    def __float__(self):
        self.item()

    def __int__(self):
        self.item()


def _find_program(tree):
    for x in pytree.tree_leaves(tree):
        if isinstance(x, SymTensor):
            return x._program
    return None


def _has_sym(tree):
    return any(isinstance(x, SymTensor) for x in pytree.tree_leaves(tree))


def _to_meta(x):
    if isinstance(x, SymTensor):
        return x.as_subclass(torch.Tensor)
    if isinstance(x, torch.Tensor) and x.device.type != "meta":
        return torch.empty_like(x, device="meta").requires_grad_(x.requires_grad)
    return x


class VarRef:
    """Placeholder for a symbolic input inside a recorded op."""

    __slots__ = ("vid",)

    def __init__(self, vid):
        self.vid = vid

    def __repr__(self):
        return f"%{self.vid}"


class Op:
    __slots__ = ("kind", "fn", "args", "kwargs", "outs", "attrs")

    def __init__(self, kind, fn, args, kwargs, outs, attrs=None):
        self.kind, self.fn, self.args, self.kwargs, self.outs = kind, fn, args, kwargs, outs
        self.attrs = attrs or {}

    @property
    def name(self):
        f = self.fn
        return getattr(f, "__qualname__", None) or getattr(f, "__name__", None) or self.kind

    def __repr__(self):
        short = lambda x: f"Tensor{list(x.shape)}" if isinstance(x, torch.Tensor) else x  # noqa: E731
        a = pytree.tree_map(short, self.args)
        k = pytree.tree_map(short, self.kwargs)
        if self.kind not in ("torch", "native"):
            return f"{self.kind}({ {k2: v for k2, v in self.attrs.items() if k2 != 'optimizer'} })"
        return f"{self.outs} = {self.name}{tuple(a)}{'' if not k else ' ' + str(k)}"


class Program:
    """paddle.static.Program: a recorded op list plus its feed (data) variables."""

    def __init__(self):
        self.ops = []
        self.feeds = {}        # name -> SymTensor
        self.vars = {}         # vid -> SymTensor (weakly the build-time handles)
        self.random_seed = 0
        self._is_test = False

    # ---------------------------------------------------------------- recording
    def new_var(self, meta, name=None):
        v = SymTensor(meta, self, name=name)
        self.vars[v._vid] = v
        return v

    def _record(self, fn, args, kwargs, kind="torch"):
        margs = pytree.tree_map(_to_meta, args)
        mkw = pytree.tree_map(_to_meta, kwargs)
        _state.recording_off += 1
        try:
            with torch._C.DisableTorchFunctionSubclass():
                out = fn(*margs, **mkw)
        finally:
            _state.recording_off -= 1
        ref = lambda x: VarRef(x._vid) if isinstance(x, SymTensor) else x  # noqa: E731
        rargs = pytree.tree_map(ref, args)
        rkw = pytree.tree_map(ref, kwargs)
        # in-place ops return their (symbolic) first argument: keep its id
        first = args[0] if args else None
        m0 = margs[0] if margs else None
        outs = []

        def wrap(t):
            if isinstance(t, torch.Tensor) and t.device.type == "meta":
                if isinstance(first, SymTensor) and t is m0:
                    outs.append(first._vid)
                    return first
                v = self.new_var(t)
                outs.append(v._vid)
                return v
            outs.append(None)
            return t

        res = pytree.tree_map(wrap, out)
        if any(o is not None for o in outs):  # pure metadata queries (dim, shape, ...) are not ops
            self.ops.append(Op(kind, fn, rargs, rkw, outs,
                               {"op_device": _state.op_device} if _state.op_device else None))
        return res

    def append_special(self, kind, **attrs):
        self.ops.append(Op(kind, None, (), {}, [], attrs))

    # ---------------------------------------------------------------- Paddle API
    def global_block(self):
        return self

    def block(self, idx=0):
        return self

    @property
    def num_blocks(self):
        return 1

    def clone(self, for_test=False):
        p = Program()
        p.ops = [o for o in self.ops if not (for_test and o.kind in ("backward", "optimize", "grad", "param_grad"))]
        p.feeds = dict(self.feeds)
        p.vars = dict(self.vars)
        p._is_test = for_test
        return p

    def all_parameters(self):
        from ..framework.param import Parameter

        seen, out = set(), []
        for o in self.ops:
            for x in pytree.tree_leaves((o.args, o.kwargs)):
                if isinstance(x, torch.Tensor) and getattr(x, "_pd_param", None) is not None and id(x) not in seen:
                    seen.add(id(x))
                    out.append(x._pd_param)
        return out

    def list_vars(self):
        return list(self.vars.values())

    def __repr__(self):
        lines = [f"Program(feeds={list(self.feeds)}, ops={len(self.ops)})"]
        for o in self.ops[:200]:
            lines.append("  " + repr(o))
        return "\n".join(lines)

    to_string = lambda self, throw_on_error=True, with_details=False: repr(self)  # noqa: E731


_main = Program()
_startup = Program()
_stack = []


def default_main_program():
    return _stack[-1][0] if _stack else _main


def default_startup_program():
    return _stack[-1][1] if _stack else _startup


@contextlib.contextmanager
def program_guard(main_program, startup_program=None):
    _stack.append((main_program, startup_program or Program()))
    try:
        yield
    finally:
        _stack.pop()


def graph_op(fn):
    """Record a whole native-kernel entry point as ONE op when it is called on symbolic tensors."""

    @functools.wraps(fn)
    def w(*args, **kwargs):
        if _state.recording_off or not _has_sym((args, kwargs)):
            return fn(*args, **kwargs)
        prog = _find_program((args, kwargs))
        return prog._record(fn, args, kwargs, kind="native")

    w._graph_op = True
    return w
