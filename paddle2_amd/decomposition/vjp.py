"""Reverse-mode differentiation of a decomposed PIR program through per-primitive VJP rules (reference:
paddle/fluid/primitive/rule/vjp/details.h — the composite backward rules — and python/paddle/autograd/ir_backward.py
``append_backward`` / ``grad`` on PIR).

``append_backward(program, out, inputs, out_grad=None)`` walks the ops that ``out`` depends on in reverse order and
emits, for every primitive, the primitive ops of its vector-Jacobian product; gradients of a value used several times
are summed, broadcast operands get their gradient reduced back to their own shape.  The backward ops are inserted in
front of the program's fetch ops, so ``pir.run`` executes forward and backward in one pass.  Composite ops must be
decomposed first (``decomposition.decompose``): an op without a VJP rule raises.
"""
from __future__ import annotations

import math

import torch

from . import rules as R


class _B:
    """Builder inserting in front of ``anchor`` (None = append)."""

    def __init__(self, program, anchor):
        self.p, self.anchor = program, anchor

    def _put(self, o):
        if self.anchor is None:
            self.p.block.append(o)
        else:
            self.p.block.insert_before(self.anchor, o)
        return o.result(0)

    def op(self, name, operands, like, **attrs):
        from ..pir import Operation

        return self._put(Operation(name, operands, [(None if like.shape is None else list(like.shape), like.dtype)],
                                   attrs))

    def op2(self, name, operands, rshape, rdtype, **attrs):
        from ..pir import Operation

        return self._put(Operation(name, operands, [(None if rshape is None else list(rshape), rdtype)], attrs))

    def reduce(self, name, x, axes):
        shape = [1 if i in axes else s for i, s in enumerate(x.shape)]
        return self.op2(name, [x], shape, x.dtype, axis=list(axes), keepdim=True)


def _unbroadcast(b, g, shape):
    """Sum g over the axes broadcasting added to reach g's shape -> a value of `shape`."""
    if list(g.shape) == list(shape):
        return g
    lead = len(g.shape) - len(shape)
    axes = list(range(lead)) + [lead + i for i, s in enumerate(shape) if s == 1 and g.shape[lead + i] != 1]
    r = b.reduce("pd_op.sum", g, axes) if axes else g
    return R.reshape(b, r, list(shape))


def _expand(b, g, shape):
    if list(g.shape) == list(shape):
        return g
    return b.op2("pd_op.expand", [g], list(shape), g.dtype, shape=list(shape))


def _float(v):
    return v.dtype in (torch.float32, torch.float64, torch.float16, torch.bfloat16)


# ------------------------------------------------------------------------------------ VJP rules: (b, op, g) -> grads
def _v_add(b, op, g):
    x, y = op.operands()
    return [_unbroadcast(b, g, x.shape), _unbroadcast(b, g, y.shape)]


def _v_sub(b, op, g):
    x, y = op.operands()
    return [_unbroadcast(b, g, x.shape), _unbroadcast(b, R.sc(b, g, -1.0), y.shape)]


def _v_mul(b, op, g):
    x, y = op.operands()
    return [_unbroadcast(b, R.mul(b, g, y), x.shape), _unbroadcast(b, R.mul(b, g, x), y.shape)]


def _v_div(b, op, g):
    x, y = op.operands()
    out = op.result(0)
    gx = R.div(b, g, y)
    gy = R.sc(b, R.div(b, R.mul(b, g, out), y), -1.0)
    return [_unbroadcast(b, gx, x.shape), _unbroadcast(b, gy, y.shape)]


def _v_minmax(name):
    def rule(b, op, g):
        x, y = op.operands()
        pick_x = R.cmp(b, name, x, y)     # x strictly wins; ties go to y
        zero = R.full(b, g.shape, 0.0, g.dtype)
        return [_unbroadcast(b, R.where(b, pick_x, g, zero), x.shape),
                _unbroadcast(b, R.where(b, pick_x, zero, g), y.shape)]
    return rule


def _v_scale(b, op, g):
    return [R.sc(b, g, op.attrs().get("scale", 1.0))]


def _v_exp(b, op, g):
    return [R.mul(b, g, op.result(0))]


def _v_log(b, op, g):
    return [R.div(b, g, op.operand_source(0))]


def _v_tanh(b, op, g):
    t = op.result(0)
    return [R.mul(b, g, R.sc(b, R.mul(b, t, t), -1.0, 1.0))]


def _v_sigmoid(b, op, g):
    s = op.result(0)
    return [R.mul(b, g, R.mul(b, s, R.sc(b, s, -1.0, 1.0)))]


def _v_erf(b, op, g):
    x = op.operand_source(0)
    d = R.sc(b, R.un(b, "pd_op.exp", R.sc(b, R.mul(b, x, x), -1.0)), 2.0 / math.sqrt(math.pi))
    return [R.mul(b, g, d)]


def _v_rsqrt(b, op, g):
    r = op.result(0)
    return [R.mul(b, g, R.sc(b, R.mul(b, R.mul(b, r, r), r), -0.5))]


def _v_sqrt(b, op, g):
    return [R.div(b, R.sc(b, g, 0.5), op.result(0))]


def _v_abs(b, op, g):
    return [R.mul(b, g, R.un(b, "pd_op.sign", op.operand_source(0)))]


def _v_pow(b, op, g):
    x = op.operand_source(0)
    y = float(op.attrs()["y"])
    return [R.mul(b, g, R.sc(b, b.op("pd_op.pow", [x], x, y=y - 1.0), y))]


def _v_sum(b, op, g):
    x = op.operand_source(0)
    return [_expand(b, g, x.shape)]


def _v_max(b, op, g):
    # the gradient is shared by every position holding the extremum (ties split evenly, as torch.amax)
    x, out = op.operand_source(0), op.result(0)
    hit = R.cast(b, R.cmp(b, "pd_op.equal", x, _expand(b, out, x.shape)), g.dtype)
    cnt = b.reduce("pd_op.sum", hit, op.attrs()["axis"])
    return [R.mul(b, hit, _expand(b, R.div(b, g, cnt), x.shape))]


def _v_reshape(b, op, g):
    return [R.reshape(b, g, op.operand_source(0).shape)]


def _v_expand(b, op, g):
    return [_unbroadcast(b, g, op.operand_source(0).shape)]


def _v_transpose(b, op, g):
    perm = list(op.attrs()["perm"])
    inv = [perm.index(i) for i in range(len(perm))]
    x = op.operand_source(0)
    return [b.op2("pd_op.transpose", [g], x.shape, g.dtype, perm=inv)]


def _v_concat(b, op, g):
    axis = op.attrs()["axis"]
    out, start = [], 0
    for x in op.operands():
        n = x.shape[axis]
        out.append(b.op2("pd_op.slice", [g], x.shape, g.dtype, axis=axis, start=start, end=start + n))
        start += n
    return out


def _v_slice(b, op, g):
    x = op.operand_source(0)
    at = op.attrs()
    axis, s, e = at["axis"], at["start"], at["end"]
    parts = []
    if s > 0:
        parts.append(R.full(b, [s if i == axis else d for i, d in enumerate(x.shape)], 0.0, g.dtype))
    parts.append(g)
    if e < x.shape[axis]:
        parts.append(R.full(b, [x.shape[axis] - e if i == axis else d for i, d in enumerate(x.shape)], 0.0, g.dtype))
    if len(parts) == 1:
        return [g]
    return [b.op2("pd_op.concat", parts, x.shape, g.dtype, axis=axis)]


def _v_gather(b, op, g):
    x, idx = op.operands()
    zero = R.full(b, x.shape, 0.0, g.dtype)
    return [b.op2("pd_op.index_add", [zero, idx, g], x.shape, g.dtype, axis=op.attrs()["axis"]), None]


def _v_take_along(b, op, g):
    x, idx = op.operands()
    zero = R.full(b, x.shape, 0.0, g.dtype)
    return [b.op2("pd_op.scatter_add_along", [zero, idx, g], x.shape, g.dtype, axis=op.attrs()["axis"]), None]


def _v_matmul(b, op, g):
    x, y = op.operands()
    at = op.attrs()
    tx, ty = bool(at.get("transpose_x")), bool(at.get("transpose_y"))

    def mm(a, c, ta, tc, shape):
        return b.op2("pd_op.matmul", [a, c], shape, g.dtype, transpose_x=ta, transpose_y=tc)

    def full_shape(v, other, g_):
        return list(g_.shape[:-2]) + list(v.shape[-2:])

    # x (after optional transpose) [.., m, k] . y [.., k, n] = g [.., m, n]
    # with A = op_x(x), B = op_y(y): dA = g B^T, dB = A^T g; dx = dA or dA^T, dy = dB or dB^T
    gx = mm(y, g, ty, True, full_shape(x, y, g)) if tx else mm(g, y, False, not ty, full_shape(x, y, g))
    gy = mm(g, x, True, tx, full_shape(y, x, g)) if ty else mm(x, g, not tx, False, full_shape(y, x, g))
    return [_unbroadcast(b, gx, x.shape), _unbroadcast(b, gy, y.shape)]


def _v_cast(b, op, g):
    x = op.operand_source(0)
    return [R.cast(b, g, x.dtype) if _float(x) else None]


def _v_where(b, op, g):
    c, x, y = op.operands()
    zero = R.full(b, g.shape, 0.0, g.dtype)
    return [None, _unbroadcast(b, R.where(b, c, g, zero), x.shape), _unbroadcast(b, R.where(b, c, zero, g), y.shape)]


def _v_index_add(b, op, g):
    x, idx, src = op.operands()
    gs = b.op2("pd_op.gather", [g, idx], src.shape, g.dtype, axis=op.attrs()["axis"])
    return [g, None, gs]


def _v_none(b, op, g):
    return [None] * op.num_operands()


VJP = {
    "pd_op.add": _v_add, "pd_op.subtract": _v_sub, "pd_op.multiply": _v_mul, "pd_op.divide": _v_div,
    "pd_op.maximum": _v_minmax("pd_op.greater_than"), "pd_op.minimum": _v_minmax("pd_op.less_than"),
    "pd_op.scale": _v_scale, "pd_op.exp": _v_exp, "pd_op.log": _v_log, "pd_op.tanh": _v_tanh,
    "pd_op.sigmoid": _v_sigmoid, "pd_op.erf": _v_erf, "pd_op.rsqrt": _v_rsqrt, "pd_op.sqrt": _v_sqrt,
    "pd_op.abs": _v_abs, "pd_op.pow": _v_pow, "pd_op.sum": _v_sum, "pd_op.max": _v_max, "pd_op.min": _v_max,
    "pd_op.reshape": _v_reshape, "pd_op.expand": _v_expand, "pd_op.transpose": _v_transpose,
    "pd_op.concat": _v_concat, "pd_op.slice": _v_slice, "pd_op.gather": _v_gather,
    "pd_op.take_along_axis": _v_take_along, "pd_op.matmul": _v_matmul, "pd_op.cast": _v_cast,
    "pd_op.where": _v_where, "pd_op.index_add": _v_index_add,
    # no gradient: comparisons, constants, sign / floor, random
    "pd_op.greater_than": _v_none, "pd_op.greater_equal": _v_none, "pd_op.less_than": _v_none,
    "pd_op.less_equal": _v_none, "pd_op.equal": _v_none, "pd_op.not_equal": _v_none, "pd_op.sign": _v_none,
    "pd_op.floor": _v_none, "pd_op.full": _v_none, "pd_op.arange": _v_none, "pd_op.uniform": _v_none,
}


_ELEMENTWISE = {"pd_op.add", "pd_op.subtract", "pd_op.multiply", "pd_op.divide", "pd_op.maximum", "pd_op.minimum"}
_UNARY = {"pd_op.exp", "pd_op.log", "pd_op.tanh", "pd_op.sigmoid", "pd_op.sqrt", "pd_op.rsqrt", "pd_op.abs",
          "pd_op.erf"}


def canonicalize(program):
    """Rewrite translated ProgramDesc ops whose semantics ARE a primitive's (matmul with trans flags, numpy-broadcast
    elementwise ops, unary math, scale, static reshape, transpose) into the primitive form the VJP rules and the
    interpreter's primitive table read.  Returns the number of ops rewritten."""
    n = 0
    for o in program.block.ops:
        at = o.attrs_
        if "__slots__" not in at:
            continue
        name = o.name()
        if name == "pd_op.matmul" and o.num_operands() == 2:
            new = {"transpose_x": bool(at.get("trans_x", at.get("transpose_X", False))),
                   "transpose_y": bool(at.get("trans_y", at.get("transpose_Y", False)))}
        elif name in _ELEMENTWISE and o.num_operands() == 2 and at.get("axis", -1) in (-1, None):
            a, c = o.operands()
            if a.shape is None or c.shape is None or (len(c.shape) > len(a.shape) and at.get("axis", -1) != -1):
                continue
            new = {}
        elif name in _UNARY and o.num_operands() == 1 and o.num_results() == 1:
            new = {}
        elif name == "pd_op.scale" and o.num_operands() == 1:
            sc_, bias = float(at.get("scale", 1.0)), float(at.get("bias", 0.0))
            new = {"scale": sc_, "bias": bias if at.get("bias_after_scale", True) else bias * sc_}
        elif name == "pd_op.reshape" and R._static(o.result(0)) and all(r.use_empty() for r in o.results()[1:]):
            new = {"shape": list(o.result(0).shape)}
        elif name == "pd_op.transpose" and "axis" in at and all(r.use_empty() for r in o.results()[1:]):
            new = {"perm": list(at["axis"])}
        else:
            continue
        o.attrs_ = new
        n += 1
    return n


def append_backward(program, out, inputs, out_grad=None):
    """Append the backward of ``out`` (a Value of ``program``) w.r.t. ``inputs`` (Values) as primitive ops; returns
    the gradient Values (None for an input ``out`` does not depend on).  ``out_grad`` defaults to ones."""
    blk = program.block
    canonicalize(program)
    anchor = next((o for o in blk.ops if o.name() == "pd_op.fetch"), None)
    b = _B(program, anchor)
    fwd_ops = [o for o in blk.ops if o is not anchor and o.name() != "pd_op.fetch"]
    # ops `out` depends on
    needed, live = set(), {out.id}
    for o in reversed(fwd_ops):
        if any(r.id in live for r in o.results()):
            needed.add(id(o))
            live.update(v.id for v in o.operands())
    grads = {out.id: out_grad if out_grad is not None else R.full(b, out.shape, 1.0, out.dtype)}
    for o in reversed(fwd_ops):
        if id(o) not in needed or o.name() in ("pd_op.data", "builtin.parameter"):
            continue
        g = grads.get(o.result(0).id)
        if g is None:
            continue
        rule = VJP.get(o.name())
        if rule is None or "__slots__" in o.attrs_:
            raise NotImplementedError(f"no primitive VJP for {o.name()} — decompose the program first")
        for v, gv in zip(o.operands(), rule(b, o, g)):
            if gv is None or not _float(v):
                continue
            prev = grads.get(v.id)
            grads[v.id] = gv if prev is None else R.add(b, prev, gv)
    return [grads.get(v.id) for v in inputs]


def add_fetch(program, values):
    """Fetch extra Values (e.g. the gradients) after the existing fetches; returns their fetch columns."""
    from ..pir import Operation

    col = sum(1 for o in program.block.ops if o.name() == "pd_op.fetch")
    cols = []
    for v in values:
        program.block.append(Operation("pd_op.fetch", [v], [(v.shape, v.dtype)], {"name": f"grad_{v.id}", "col": col}))
        cols.append(col)
        col += 1
    return cols
