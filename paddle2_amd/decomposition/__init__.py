"""Primitive decomposition of composite ops on PIR programs (reference: paddle/fluid/primitive/ composite rules
and python/paddle/decomposition/decomp.py ``decompose``).

Composite ops are rewritten into a small primitive set — exp, log, erf, tanh, rsqrt, sigmoid, max / sum
reductions (keepdim), add / subtract / multiply / divide / maximum / minimum and scale (``scale(x, 0, c)`` is the
constant-like-x primitive) — which compiler-style passes (and the interpreter) handle uniformly.  Rules:
softmax, log_softmax, gelu (erf and tanh forms), silu / swish, mish, softplus, relu, relu6, leaky_relu, elu,
hardswish, hardsigmoid, square, reciprocal, swiglu, rms_norm, layer_norm (when its Mean / Variance side outputs
are unused), mean and logsumexp here; the rest of the reference's composite set (norms, losses, shape ops,
embedding, dropout, more activations) in ``decomposition.rules``.  ``decomposition.vjp.append_backward`` then
differentiates a decomposed program through per-primitive VJP rules (reference
paddle/fluid/primitive/rule/vjp/details.h)."""
from __future__ import annotations

import math

from ..pir import Operation

PRIMITIVES = {"pd_op.exp", "pd_op.log", "pd_op.erf", "pd_op.rsqrt", "pd_op.sigmoid", "pd_op.max", "pd_op.sum",
              "pd_op.add", "pd_op.subtract", "pd_op.multiply", "pd_op.divide", "pd_op.maximum", "pd_op.minimum",
              "pd_op.scale", "pd_op.tanh"}


class _Builder:
    def __init__(self, program, anchor):
        self.p, self.anchor = program, anchor

    def op(self, name, operands, like, **attrs):
        o = Operation(name, operands, [(list(like.shape) if like.shape is not None else None, like.dtype)], attrs)
        self.p.block.insert_before(self.anchor, o)
        return o.result(0)

    def op2(self, name, operands, rshape, rdtype, **attrs):
        o = Operation(name, operands, [(None if rshape is None else list(rshape), rdtype)], attrs)
        self.p.block.insert_before(self.anchor, o)
        return o.result(0)

    def reduce(self, name, x, axes):
        shape = None if x.shape is None else [1 if i in axes else s for i, s in enumerate(x.shape)]
        o = Operation(name, [x], [(shape, x.dtype)], {"axis": list(axes), "keepdim": True})
        self.p.block.insert_before(self.anchor, o)
        return o.result(0)


def _axes(x, axis):
    nd = len(x.shape)
    return [axis % nd]


def _softmax(b, op, log=False):
    x = op.operand_source(0)
    ax = _axes(x, op.attrs().get("axis", -1))
    m = b.reduce("pd_op.max", x, ax)
    s = b.op("pd_op.subtract", [x, m], x)
    e = b.op("pd_op.exp", [s], x)
    z = b.reduce("pd_op.sum", e, ax)
    if log:
        return b.op("pd_op.subtract", [s, b.op("pd_op.log", [z], z)], x)
    return b.op("pd_op.divide", [e, z], x)


def _const(b, like, c):
    """A tensor shaped like ``like`` filled with c: scale(like, 0, c)."""
    return b.op("pd_op.scale", [like], like, scale=0.0, bias=float(c))


def _relu(b, op):
    x = op.operand_source(0)
    return b.op("pd_op.maximum", [x, _const(b, x, 0.0)], x)


def _relu6(b, op):
    x = op.operand_source(0)
    r = b.op("pd_op.maximum", [x, _const(b, x, 0.0)], x)
    return b.op("pd_op.minimum", [r, _const(b, x, op.attrs().get("threshold", 6.0))], x)


def _leaky_relu(b, op):
    x = op.operand_source(0)
    a = float(op.attrs().get("alpha", 0.02))
    ax = b.op("pd_op.scale", [x], x, scale=a, bias=0.0)
    return b.op("pd_op.maximum" if a <= 1.0 else "pd_op.minimum", [x, ax], x)


def _elu(b, op):
    x = op.operand_source(0)
    a = float(op.attrs().get("alpha", 1.0))
    zero = _const(b, x, 0.0)
    neg = b.op("pd_op.scale", [b.op("pd_op.exp", [b.op("pd_op.minimum", [x, zero], x)], x)], x, scale=a, bias=-a)
    return b.op("pd_op.add", [b.op("pd_op.maximum", [x, zero], x), neg], x)


def _softplus_of(b, x, beta=1.0, threshold=20.0):
    # log(1 + exp(beta x)) / beta, computed stably as max(bx, 0) + log(1 + exp(-|bx|))
    bx = b.op("pd_op.scale", [x], x, scale=beta, bias=0.0)
    zero = _const(b, x, 0.0)
    pos = b.op("pd_op.maximum", [bx, zero], x)
    nabs = b.op("pd_op.minimum", [bx, b.op("pd_op.scale", [bx], x, scale=-1.0, bias=0.0)], x)
    l1p = b.op("pd_op.log", [b.op("pd_op.scale", [b.op("pd_op.exp", [nabs], x)], x, scale=1.0, bias=1.0)], x)
    sp = b.op("pd_op.add", [pos, l1p], x)
    return sp if beta == 1.0 else b.op("pd_op.scale", [sp], x, scale=1.0 / beta, bias=0.0)


def _softplus(b, op):
    return _softplus_of(b, op.operand_source(0), float(op.attrs().get("beta", 1.0)))


def _mish(b, op):
    x = op.operand_source(0)
    return b.op("pd_op.multiply", [x, b.op("pd_op.tanh", [_softplus_of(b, x)], x)], x)


def _hardsigmoid_of(b, x, slope, offset):
    y = b.op("pd_op.scale", [x], x, scale=slope, bias=offset)
    return b.op("pd_op.minimum", [b.op("pd_op.maximum", [y, _const(b, x, 0.0)], x), _const(b, x, 1.0)], x)


def _hardsigmoid(b, op):
    at = op.attrs()
    return _hardsigmoid_of(b, op.operand_source(0), float(at.get("slope", 0.1666667)), float(at.get("offset", 0.5)))


def _hardswish(b, op):
    x = op.operand_source(0)
    return b.op("pd_op.multiply", [x, _hardsigmoid_of(b, x, 1.0 / 6.0, 0.5)], x)


def _square(b, op):
    x = op.operand_source(0)
    return b.op("pd_op.multiply", [x, x], x)


def _reciprocal(b, op):
    x = op.operand_source(0)
    return b.op("pd_op.divide", [_const(b, x, 1.0), x], x)


def _swiglu(b, op):
    # swiglu(x, y) = silu(x) * y; single-operand form splits the last axis in halves (not decomposed here)
    if op.num_operands() != 2:
        return None
    x, y = op.operand_source(0), op.operand_source(1)
    return b.op("pd_op.multiply", [b.op("pd_op.multiply", [x, b.op("pd_op.sigmoid", [x], x)], x), y], x)


def _rms_norm(b, op):
    if any(not r.use_empty() for r in op.results()[1:]):
        return None
    x = op.operand_source(0)
    axes = [len(x.shape) - 1]
    n = x.shape[-1]
    ms = b.op("pd_op.scale", [b.reduce("pd_op.sum", b.op("pd_op.multiply", [x, x], x), axes)],
              b.reduce("pd_op.sum", x, axes), scale=1.0 / n, bias=float(op.attrs().get("epsilon", 1e-6)))
    y = b.op("pd_op.multiply", [x, b.op("pd_op.rsqrt", [ms], ms)], x)
    if op.num_operands() > 1:
        y = b.op("pd_op.multiply", [y, op.operand_source(1)], x)
    return y


def _reduce_axes(op, x):
    at = op.attrs()
    nd = len(x.shape)
    if at.get("reduce_all") or not at.get("dim", at.get("axis")):
        return list(range(nd))
    ax = at.get("dim", at.get("axis"))
    ax = ax if isinstance(ax, (list, tuple)) else [ax]
    return sorted(a % nd for a in ax)


def _mean(b, op):
    x = op.operand_source(0)
    if op.num_operands() != 1 or x.shape is None or any(s is None or s < 0 for s in x.shape):
        return None
    axes = _reduce_axes(op, x)
    if not op.attrs().get("keep_dim", op.attrs().get("keepdim", False)) and len(axes) != len(x.shape):
        return None   # the primitive reductions keep dims; a squeeze would be needed
    n = 1
    for a in axes:
        n *= x.shape[a]
    s = b.reduce("pd_op.sum", x, axes)
    return b.op("pd_op.scale", [s], s, scale=1.0 / n, bias=0.0)


def _logsumexp(b, op):
    x = op.operand_source(0)
    axes = _reduce_axes(op, x)
    if not op.attrs().get("keepdim", False):
        return None
    m = b.reduce("pd_op.max", x, axes)
    z = b.reduce("pd_op.sum", b.op("pd_op.exp", [b.op("pd_op.subtract", [x, m], x)], x), axes)
    return b.op("pd_op.add", [m, b.op("pd_op.log", [z], z)], m)


def _gelu(b, op):
    x = op.operand_source(0)
    if op.attrs().get("approximate"):
        x3 = b.op("pd_op.multiply", [b.op("pd_op.multiply", [x, x], x), x], x)
        inner = b.op("pd_op.add", [x, b.op("pd_op.scale", [x3], x, scale=0.044715, bias=0.0)], x)
        t = b.op("pd_op.tanh", [b.op("pd_op.scale", [inner], x, scale=math.sqrt(2.0 / math.pi), bias=0.0)], x)
    else:
        t = b.op("pd_op.erf", [b.op("pd_op.scale", [x], x, scale=1.0 / math.sqrt(2.0), bias=0.0)], x)
    one_plus = b.op("pd_op.scale", [t], x, scale=1.0, bias=1.0)
    return b.op("pd_op.scale", [b.op("pd_op.multiply", [x, one_plus], x)], x, scale=0.5, bias=0.0)


def _silu(b, op):
    x = op.operand_source(0)
    return b.op("pd_op.multiply", [x, b.op("pd_op.sigmoid", [x], x)], x)


def _layer_norm(b, op):
    if any(not r.use_empty() for r in op.results()[1:]):
        return None
    x = op.operand_source(0)
    slots = op.attrs().get("__slots__", ["X", "Scale", "Bias"])
    ops = dict(zip(slots, op.operands()))
    nd = len(x.shape)
    axes = list(range(op.attrs().get("begin_norm_axis", 1), nd))
    n = 1
    for a in axes:
        n *= x.shape[a]
    mean = b.op("pd_op.scale", [b.reduce("pd_op.sum", x, axes)], b.reduce("pd_op.sum", x, axes), scale=1.0 / n,
                bias=0.0)
    xc = b.op("pd_op.subtract", [x, mean], x)
    var = b.op("pd_op.scale", [b.reduce("pd_op.sum", b.op("pd_op.multiply", [xc, xc], x), axes)], mean,
               scale=1.0 / n, bias=0.0)
    rstd = b.op("pd_op.rsqrt", [b.op("pd_op.scale", [var], var, scale=1.0, bias=op.attrs().get("epsilon", 1e-5))],
                var)
    y = b.op("pd_op.multiply", [xc, rstd], x)
    if "Scale" in ops:
        y = b.op("pd_op.multiply", [y, ops["Scale"]], x)
    if "Bias" in ops:
        y = b.op("pd_op.add", [y, ops["Bias"]], x)
    return y


_RULES = {"pd_op.softmax": _softmax, "pd_op.log_softmax": lambda b, op: _softmax(b, op, log=True),
          "pd_op.gelu": _gelu, "pd_op.silu": _silu, "pd_op.swish": _silu, "pd_op.layer_norm": _layer_norm,
          "pd_op.relu": _relu, "pd_op.relu6": _relu6, "pd_op.leaky_relu": _leaky_relu, "pd_op.elu": _elu,
          "pd_op.softplus": _softplus, "pd_op.mish": _mish, "pd_op.hardsigmoid": _hardsigmoid,
          "pd_op.hardswish": _hardswish, "pd_op.square": _square, "pd_op.reciprocal": _reciprocal,
          "pd_op.swiglu": _swiglu, "pd_op.rms_norm": _rms_norm, "pd_op.mean": _mean, "pd_op.logsumexp": _logsumexp}


from .rules import EXTRA_PRIMITIVES as _EXTRA, RULES as _MORE  # noqa: E402

_RULES.update(_MORE)
PRIMITIVES = PRIMITIVES | _EXTRA


def has_rule(name):
    return name in _RULES


def decompose(program, src_vars=None, blacklist=frozenset(), whitelist=frozenset()):
    """Rewrite every composite op with a rule (restricted to ``whitelist`` if given, minus ``blacklist``).
    Returns the number of ops decomposed."""
    n = 0
    for op in list(program.block.ops):
        name = op.name()
        rule = _RULES.get(name)
        if rule is None or name in blacklist or (whitelist and name not in whitelist):
            continue
        new = rule(_Builder(program, op), op)
        if new is None:
            continue
        if isinstance(new, (list, tuple)):   # multi-output op (unbind / unstack / meshgrid): one value per result
            for i, v in enumerate(new):
                op.result(i).replace_all_uses_with(v)
        else:
            op.result(0).replace_all_uses_with(new)
        program.block.remove_op(op)
        n += 1
    return n
