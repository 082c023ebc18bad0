"""PIR as the executed IR of the static Executor (reference: paddle/fluid/framework/new_executor/pir_interpreter.cc —
the new executor runs a PIR program after the pass pipeline; python/paddle/base/executor.py `_run_pir_impl`).

``Executor.run`` no longer replays the recorded op list as recorded: the Program is translated into SSA form
(``from_recorded``), the PIR pass pipeline runs on it (dead-code elimination against the fetch targets and every
side-effecting instruction, common-subexpression elimination of pure ops, fused_gemm_epilogue), and the optimised
PIR is lowered back to instructions (``to_recorded``) from which csrc/runtime/interpreter.cpp builds the dependency /
stream / GC plan the Executor issues.  So what executes is the PIR after its passes.

Translation: every recorded instruction becomes one Operation.  Recognised torch / native ops get their pd_op
names (matmul, add, multiply, relu, gelu, linear, ...) so the passes can pattern-match them; the rest keep a
``rec.<kind>.<function>`` name.  Tensor operands are Values: symbolic variables (feeds ``pd_op.data``, op results)
and captured real tensors (parameters, buffers, constants: ``builtin.parameter``); non-tensor arguments stay in
the op's argument template.  In-place instructions, backward / grad / optimizer instructions and in-place
methods on captured tensors are side effects: DCE keeps them and CSE never merges them.
"""
from __future__ import annotations

import torch
from torch.utils import _pytree as pytree

from . import Operation, Program

_RANDOM = ("dropout", "rand", "randn", "randint", "bernoulli", "multinomial", "normal", "uniform", "gaussian",
           "randperm", "native_dropout")


class _Opnd:
    __slots__ = ("i",)

    def __init__(self, i):
        self.i = i

    def __repr__(self):
        return f"$${self.i}"


def _fn_name(op):
    f = op.fn
    return getattr(f, "__name__", None) or getattr(f, "__qualname__", None) or op.kind


def _pd_name(op):
    """pd_op name of a recorded instruction (for the pattern passes), or rec.<kind>.<fn>."""
    if op.kind not in ("torch", "native"):
        return "rec." + op.kind
    n = _fn_name(op)
    q = getattr(op.fn, "__qualname__", "") or ""
    table = {"matmul": "matmul", "mm": "matmul", "add": "add", "__add__": "add", "sub": "subtract",
             "__sub__": "subtract", "mul": "multiply", "__mul__": "multiply", "div": "divide",
             "__truediv__": "divide", "relu": "relu", "gelu": "gelu", "linear": "linear", "addmm": "addmm",
             "exp": "exp", "tanh": "tanh", "sigmoid": "sigmoid", "neg": "neg", "rsqrt": "rsqrt"}
    base = table.get(n)
    if base is not None and (op.kind == "torch" or n == "linear"):
        return "pd_op." + base
    return f"rec.{op.kind}.{q or n}"


def _known_pure_fn(fn):
    """torch operators and the framework's kernel entry points (ops/, pir/kernels.py) compute their outputs from
    their inputs; any other recorded callable (a send / recv, a user hook, ...) may act outside the program."""
    mod = getattr(fn, "__module__", None)
    if mod is None:   # builtin methods of torch._C.TensorBase / VariableFunctions
        owner = getattr(fn, "__objclass__", None) or getattr(fn, "__self__", None)
        mod = getattr(owner, "__module__", None) or type(owner).__module__
    mod = str(mod or "")
    return mod.startswith("torch") or mod.startswith("paddle2_amd.ops") or mod.startswith("paddle2_amd.pir")


def _side_effect(op, reads):
    if op.kind not in ("torch", "native"):
        return True
    if not _known_pure_fn(op.fn):
        return True
    n = _fn_name(op)
    if n.endswith("_") and not n.endswith("__"):   # in-place torch method (add_, copy_, ...)
        return True
    if n in ("__iadd__", "__isub__", "__imul__", "__itruediv__", "__ifloordiv__", "__ipow__", "__iand__",
             "__ior__", "__ixor__", "__setitem__", "__delitem__") or "out" in op.kwargs or op.kwargs.get("inplace"):
        return True
    # an op returning its input unchanged (x.long() on an int64 x, a no-op view) keeps the variable id: an alias,
    # not a write
    if op.attrs.get("stream") or getattr(op.fn, "_pd_stream", None):   # collectives / copies on side streams
        return True
    return False


def _impure(op):
    n = _fn_name(op).lower()
    return any(r in n for r in _RANDOM)


def _freeze(v):
    if isinstance(v, torch.Tensor):
        return ("tensor", id(v))
    if isinstance(v, (list, tuple)):
        return (type(v).__name__,) + tuple(_freeze(x) for x in v)
    if isinstance(v, dict):
        return ("dict",) + tuple(sorted((str(k), _freeze(x)) for k, x in v.items()))
    if isinstance(v, _Opnd):
        return ("opnd", v.i)
    try:
        hash(v)
        return v
    except TypeError:
        return ("obj", id(v))


def from_recorded(program, fetch_ids):
    """Recorded static Program -> PIR Program (see module doc)."""
    from ..static.executor import _op_reads

    pp = Program()
    env = {}           # vid -> current Value
    params = {}        # id(captured tensor) -> Value

    def meta_of(vid):
        v = program.vars.get(vid)
        return (list(v.shape), v.dtype) if v is not None else (None, torch.float32)

    for name, sym in program.feeds.items():
        op = pp.block.append(Operation("pd_op.data", [], [meta_of(sym._vid)], {"name": name}))
        op.result(0).vid = sym._vid
        env[sym._vid] = op.result(0)

    def param(t):
        v = params.get(id(t))
        if v is None:
            op = pp.block.append(Operation("builtin.parameter", [], [(list(t.shape), t.dtype)],
                                           {"parameter_name": f"captured_{len(params)}"}))
            v = op.result(0)
            v.tensor = t
            pp.params[v.id] = t
            params[id(t)] = v
        return v

    from ..static.graph import VarRef

    for rop in program.ops:
        reads = _op_reads(rop)
        operands = []

        def tpl(x):
            if isinstance(x, VarRef):
                operands.append(env[x.vid])
                return _Opnd(len(operands) - 1)
            if isinstance(x, torch.Tensor) and x.device.type != "meta":
                operands.append(param(x))
                return _Opnd(len(operands) - 1)
            return x

        args_t = pytree.tree_map(tpl, rop.args)
        kwargs_t = pytree.tree_map(tpl, rop.kwargs)
        # attribute-carried reads (backward loss, grad targets / inputs) become operands too
        extra = [v for v in reads if v not in {o.vid for o in operands if hasattr(o, "vid")}]
        for v in extra:
            if v in env:
                operands.append(env[v])
        outs = [v for v in rop.outs if v is not None]
        for k in ("out",):
            if k in rop.attrs and isinstance(rop.attrs[k], int):
                outs.append(rop.attrs[k])
        outs.extend(v for v in rop.attrs.get("outs", ()) if isinstance(v, int))
        se = _side_effect(rop, set(reads))
        attrs = {"__rec__": rop, "__tpl__": (args_t, kwargs_t), "__side_effect__": se,
                 "__impure__": _impure(rop),
                 "__cse_key__": (id(rop.fn), rop.kind, _freeze(args_t), _freeze(kwargs_t))}
        if _fn_name(rop) == "gelu":
            attrs["approximate"] = rop.kwargs.get("approximate", "none") != "none"
        op = pp.block.append(Operation(_pd_name(rop), operands, [meta_of(v) for v in outs], attrs))
        for v, r in zip(outs, op.results()):
            r.vid = v
            env[v] = r
    for i, f in enumerate(fetch_ids):
        if f in env:
            v = env[f]
            pp.block.append(Operation("pd_op.fetch", [v], [(v.shape, v.dtype)], {"col": i, "vid": f}))
    return pp


# ------------------------------------------------------------------------------------------------ passes
def dce(pp):
    """Dead-code elimination: keep fetches, side effects and everything they (transitively) read."""
    n = 0
    changed = True
    while changed:
        changed = False
        for op in list(reversed(pp.block.ops)):
            name = op.name()
            if name in ("pd_op.fetch", "pd_op.data"):
                continue
            if op.attrs_.get("__side_effect__"):
                continue
            if all(r.use_empty() for r in op.results()):
                pp.block.remove_op(op)
                if name == "builtin.parameter":
                    pp.params.pop(op.result(0).id, None)
                n += 1
                changed = True
    return n


def cse(pp):
    """Common-subexpression elimination of pure recorded ops (same function, operands and constant args)."""
    seen, n = {}, 0
    def attr_read(op):   # a result that backward / grad instructions name by variable id in their attributes
        return any(u.attrs_.get("__rec__") is not None and u.attrs_["__rec__"].kind not in ("torch", "native")
                   for r in op.results() for u, _ in r.uses)

    for op in list(pp.block.ops):
        a = op.attrs_
        if "__cse_key__" not in a or a.get("__side_effect__") or a.get("__impure__") or attr_read(op):
            continue
        key = (a["__cse_key__"], tuple(v.id for v in op.operands()))
        prev = seen.get(key)
        if prev is None or prev.num_results() != op.num_results():
            seen[key] = op
            continue
        for x, y in zip(op.results(), prev.results()):
            x.replace_all_uses_with(y)
        pp.block.remove_op(op)
        n += 1
    return n


def _single_use(v):
    return len(v.uses) == 1


def fused_gemm_epilogue(pp):
    """matmul(x, W) -> add(., b 1-D) [-> relu | gelu]  and  linear(x, W, b) -> relu | gelu   =>   one
    fused_gemm_epilogue op (the native GEMM + the fused bias-activation kernel: reference
    paddle/fluid/pir/transforms/gpu/fused_gemm_epilogue_pass.cc)."""
    n = 0
    for op in list(pp.block.ops):
        if op.block is None or op not in pp.block.ops:
            continue
        name = op.name()
        if name not in ("pd_op.matmul", "pd_op.linear") or op.attrs_.get("__side_effect__"):
            continue
        rop = op.attrs_["__rec__"]
        args_t, kwargs_t = op.attrs_["__tpl__"]
        if kwargs_t or len(args_t) < 2 or not all(isinstance(a, _Opnd) for a in args_t[:2]):
            continue
        x = op.operand_source(args_t[0].i)
        w = op.operand_source(args_t[1].i)
        if w.shape is None or len(w.shape) != 2 or x.shape is None or len(x.shape) < 2:
            continue
        out = op.result(0)
        chain = [op]
        bias = None
        if name == "pd_op.linear":
            if len(args_t) > 2 and isinstance(args_t[2], _Opnd):
                bias = op.operand_source(args_t[2].i)
            elif len(args_t) > 2 and args_t[2] is not None:
                continue
        else:
            if not _single_use(out):
                continue
            add, _ = out.uses[0]
            at, kt = add.attrs_.get("__tpl__", ((), {}))
            if add.name() != "pd_op.add" or kt or len(at) != 2 or not all(isinstance(a, _Opnd) for a in at):
                continue
            if add.operand_source(at[0].i) is not out:
                continue
            b = add.operand_source(at[1].i)
            if b.shape is None or len(b.shape) != 1 or b.shape[0] != w.shape[1]:
                continue
            bias = b
            chain.append(add)
            out = add.result(0)
        act = "identity"
        if _single_use(out):
            nxt, _ = out.uses[0]
            nt, nk = nxt.attrs_.get("__tpl__", ((), {}))
            if nxt.name() in ("pd_op.relu", "pd_op.gelu") and len(nxt.operands()) == 1:
                act = "relu" if nxt.name() == "pd_op.relu" else (
                    "gelu_tanh" if nxt.attrs_.get("approximate") else "gelu")
                chain.append(nxt)
                out = nxt.result(0)
        if len(chain) == 1:
            continue   # a bare GEMM: nothing to fuse
        operands = [x, w] + ([bias] if bias is not None else [])
        fused = Operation("pd_op.fused_gemm_epilogue", operands, [(out.shape, out.dtype)],
                          {"activation": act, "trans_y": False, "__side_effect__": False,
                           "__has_bias__": bias is not None})
        pp.block.insert_before(chain[-1], fused)   # after the bias's definition: SSA order holds
        fused.result(0).vid = out.vid
        out.replace_all_uses_with(fused.result(0))
        for o in reversed(chain):
            pp.block.remove_op(o)
        n += 1
    return n


PIPELINE = (("dead_code_elimination_pass", dce), ("common_subexpression_elimination_pass", cse),
            ("fused_gemm_epilogue_pass", fused_gemm_epilogue), ("dead_code_elimination_pass#2", dce))


def run_passes(pp):
    return {name: fn(pp) for name, fn in PIPELINE}


# ------------------------------------------------------------------------------------------------ lowering
def _value_ref(v):
    from ..static.graph import VarRef

    t = getattr(v, "tensor", None)
    if t is not None:
        return t
    return VarRef(v.vid)


def to_recorded(pp, program):
    """Optimised PIR -> the instruction list the Executor plans and issues (a static Program sharing the
    original's feeds / variables)."""
    from ..static.graph import Op
    from ..static.graph import Program as StaticProgram
    from .kernels import fused_gemm_epilogue as fge_kernel

    out = StaticProgram()
    out.feeds, out.vars = program.feeds, program.vars
    from .kernels import alias

    for op in pp.block.ops:
        name = op.name()
        if name == "pd_op.fetch":
            src = op.operand_source(0)
            if getattr(src, "vid", None) != op.attrs_["vid"] or getattr(src, "tensor", None) is not None:
                out.ops.append(Op("torch", alias, (_value_ref(src),), {}, [op.attrs_["vid"]]))
            continue
        if name in ("pd_op.data", "builtin.parameter"):
            continue
        if name == "pd_op.fused_gemm_epilogue":
            ops = [_value_ref(v) for v in op.operands()]
            b = ops[2] if op.attrs_.get("__has_bias__") else None
            out.ops.append(Op("native", fge_kernel, (ops[0], ops[1], b), {"activation": op.attrs_["activation"]},
                              [op.result(0).vid]))
            continue
        rop = op.attrs_["__rec__"]
        args_t, kwargs_t = op.attrs_["__tpl__"]
        cur = op.operands()

        def fill(x):
            return _value_ref(cur[x.i]) if isinstance(x, _Opnd) else x

        args = pytree.tree_map(fill, args_t, is_leaf=lambda x: isinstance(x, _Opnd))
        kwargs = pytree.tree_map(fill, kwargs_t, is_leaf=lambda x: isinstance(x, _Opnd))
        out.ops.append(Op(rop.kind, rop.fn, args, kwargs, rop.outs, rop.attrs))
    return out


def optimize(program, fetch_ids):
    """Program -> (executable Program after the PIR pipeline, PIR program, pass statistics)."""
    pp = from_recorded(program, fetch_ids)
    stats = run_passes(pp)
    return to_recorded(pp, program), pp, stats
