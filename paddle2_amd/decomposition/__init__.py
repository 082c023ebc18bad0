"""Primitive decomposition of composite ops on PIR programs (reference: paddle/fluid/primitive/ composite rules
and python/paddle/decomposition/decomp.py ``decompose``).

Composite ops are rewritten into a small primitive set — exp, erf, rsqrt, sigmoid, max / sum reductions
(keepdim), add / subtract / multiply / divide and scale — which compiler-style passes (and the interpreter)
handle uniformly.  Rules: softmax, log_softmax, gelu (erf and tanh forms), silu, layer_norm (when its
Mean / Variance side outputs are unused), mean."""
from __future__ import annotations

import math

from ..pir import Operation

PRIMITIVES = {"pd_op.exp", "pd_op.erf", "pd_op.rsqrt", "pd_op.sigmoid", "pd_op.max", "pd_op.sum", "pd_op.add",
              "pd_op.subtract", "pd_op.multiply", "pd_op.divide", "pd_op.scale", "pd_op.tanh"}


class _Builder:
    def __init__(self, program, anchor):
        self.p, self.anchor = program, anchor

    def op(self, name, operands, like, **attrs):
        o = Operation(name, operands, [(list(like.shape) if like.shape is not None else None, like.dtype)], attrs)
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
    return b.op("pd_op.divide", [e, z], x)


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


_RULES = {"pd_op.softmax": _softmax, "pd_op.gelu": _gelu, "pd_op.silu": _silu, "pd_op.layer_norm": _layer_norm}


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
        op.result(0).replace_all_uses_with(new)
        program.block.remove_op(op)
        n += 1
    return n
