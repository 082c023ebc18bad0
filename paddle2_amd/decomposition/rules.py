"""More composite -> primitive rules (reference: paddle/fluid/primitive/composite/composite.h — any, mean_all,
p_norm, pow, huber_loss, one_hot, squared_l2_norm, bce_loss, bmm, batch_norm, stack, squeeze / unsqueeze,
add_n, full_like, dropout, heaviside, instance_norm, flatten, clip, index_select, group_norm,
sigmoid_cross_entropy_with_logits, embedding, index_sample, lerp, log_loss, kldiv_loss, softsign, numel — and
python/paddle/decomposition/rules.py for the activations).

Every rule reads its op through the PIR attribute names of the reference's ops.yaml (falling back to the
ProgramDesc names the translator carries) and needs static shapes where the rewrite reshapes; a rule returns
None to leave the op alone (dynamic shape, a side output in use, an unsupported mode).
"""
from __future__ import annotations

import math

import torch

# primitives these rules introduce beyond the base set (decomposition.PRIMITIVES)
EXTRA_PRIMITIVES = {"pd_op.sqrt", "pd_op.abs", "pd_op.sign", "pd_op.pow", "pd_op.reshape", "pd_op.concat",
                    "pd_op.gather", "pd_op.take_along_axis", "pd_op.matmul", "pd_op.cast", "pd_op.where",
                    "pd_op.greater_than", "pd_op.less_than", "pd_op.equal", "pd_op.not_equal", "pd_op.floor",
                    "pd_op.arange", "pd_op.full", "pd_op.uniform", "pd_op.expand", "pd_op.transpose", "pd_op.slice",
                    "pd_op.index_add", "pd_op.scatter_add_along", "pd_op.min", "pd_op.greater_equal",
                    "pd_op.less_equal"}


def _static(v):
    return v.shape is not None and all(isinstance(s, int) and s >= 0 for s in v.shape)


def _side_outputs_unused(op):
    return all(r.use_empty() for r in op.results()[1:])


def _numel(shape):
    n = 1
    for s in shape:
        n *= s
    return n


def _norm_axes(axis, nd):
    if axis is None or (isinstance(axis, (list, tuple)) and len(axis) == 0):
        return list(range(nd))
    ax = axis if isinstance(axis, (list, tuple)) else [axis]
    return sorted(int(a) % nd for a in ax)


def _attr(op, *names, default=None):
    at = op.attrs()
    for n in names:
        if n in at:
            return at[n]
    return default


# ----------------------------------------------------------------------------------------------- helpers (prims)
def full(b, shape, value, dtype):
    return b.op2("pd_op.full", [], list(shape), dtype, shape=list(shape), value=float(value), dtype=dtype)


def scalar_like(b, x, c):
    """A tensor of x's shape and dtype filled with c (no read of x: NaN / inf in x stay out of it)."""
    return full(b, x.shape, c, x.dtype)


def reshape(b, x, shape):
    return b.op2("pd_op.reshape", [x], list(shape), x.dtype, shape=list(shape))


def cast(b, x, dtype):
    return b.op2("pd_op.cast", [x], x.shape, dtype, dtype=dtype)


def reduce(b, name, x, axes, keepdim=True):
    r = b.reduce(name, x, axes)
    if keepdim:
        return r
    return reshape(b, r, [s for i, s in enumerate(x.shape) if i not in axes])


def bshape(x, y):
    """Broadcast result shape of two operands (None if either is unknown)."""
    if x.shape is None or y.shape is None:
        return None
    nd = max(len(x.shape), len(y.shape))
    xs = [1] * (nd - len(x.shape)) + list(x.shape)
    ys = [1] * (nd - len(y.shape)) + list(y.shape)
    return [max(a, c) for a, c in zip(xs, ys)]


def cmp(b, name, x, y):
    return b.op2(name, [x, y], bshape(x, y), torch.bool)


def where(b, c, x, y):
    return b.op2("pd_op.where", [c, x, y], x.shape, x.dtype)


def sc(b, x, s=1.0, bias=0.0):
    return b.op("pd_op.scale", [x], x, scale=float(s), bias=float(bias))


def bin_(b, name, x, y):
    out = x if len(x.shape or []) >= len(y.shape or []) else y
    shape = bshape(x, y)
    return b.op2(name, [x, y], shape if shape is not None else out.shape, out.dtype)


def add(b, x, y):
    return bin_(b, "pd_op.add", x, y)


def sub(b, x, y):
    return bin_(b, "pd_op.subtract", x, y)


def mul(b, x, y):
    return bin_(b, "pd_op.multiply", x, y)


def div(b, x, y):
    return bin_(b, "pd_op.divide", x, y)


def un(b, name, x):
    return b.op(name, [x], x)


def _channel_shape(x, axis):
    return [x.shape[axis] if i == axis else 1 for i in range(len(x.shape))]


def _norm(b, x, axes, eps):
    """(x - mean) * rsqrt(var + eps) over `axes` (biased variance, keepdim) -> (y, mean, var)."""
    n = _numel([x.shape[a] for a in axes])
    mean = sc(b, b.reduce("pd_op.sum", x, axes), 1.0 / n)
    xc = sub(b, x, mean)
    var = sc(b, b.reduce("pd_op.sum", mul(b, xc, xc), axes), 1.0 / n)
    return mul(b, xc, un(b, "pd_op.rsqrt", sc(b, var, 1.0, eps))), mean, var


# ----------------------------------------------------------------------------------------------- rules
def _any(b, op):
    x = op.operand_source(0)
    if not _static(x):
        return None
    axes = _norm_axes(_attr(op, "axis", "dim"), len(x.shape))
    r = reduce(b, "pd_op.max", cast(b, x, torch.float32), axes, bool(_attr(op, "keepdim", "keep_dim", default=False)))
    return cast(b, r, torch.bool)


def _mean_all(b, op):
    x = op.operand_source(0)
    if not _static(x):
        return None
    s = reduce(b, "pd_op.sum", x, list(range(len(x.shape))), keepdim=False)
    return sc(b, s, 1.0 / max(1, _numel(x.shape)))


def _p_norm(b, op):
    x = op.operand_source(0)
    if not _static(x) or _attr(op, "asvector", default=False):
        return None
    p = float(_attr(op, "porder", default=2.0))
    axes = [int(_attr(op, "axis", default=-1)) % len(x.shape)]
    keep = bool(_attr(op, "keepdim", default=False))
    if p == 0.0:
        nz = cast(b, cmp(b, "pd_op.not_equal", x, scalar_like(b, x, 0.0)), x.dtype)
        return reduce(b, "pd_op.sum", nz, axes, keep)
    if p == 1.0:
        return reduce(b, "pd_op.sum", un(b, "pd_op.abs", x), axes, keep)
    if p == 2.0:
        return un(b, "pd_op.sqrt", reduce(b, "pd_op.sum", mul(b, x, x), axes, keep))
    if p == math.inf:
        return reduce(b, "pd_op.max", un(b, "pd_op.abs", x), axes, keep)
    if p == -math.inf:
        return reduce(b, "pd_op.min", un(b, "pd_op.abs", x), axes, keep)
    s = reduce(b, "pd_op.sum", b.op("pd_op.pow", [un(b, "pd_op.abs", x)], x, y=p), axes, keep)
    return b.op("pd_op.pow", [s], s, y=1.0 / p)


def _pow(b, op):
    if op.num_operands() != 1:
        return None
    x = op.operand_source(0)
    y = float(_attr(op, "y", "factor", default=1.0))
    if y == 2.0:
        return mul(b, x, x)
    if y == 3.0:
        return mul(b, mul(b, x, x), x)
    if y == 0.5:
        return un(b, "pd_op.sqrt", x)
    if y == -1.0:
        return div(b, scalar_like(b, x, 1.0), x)
    if y == 1.0:
        return sc(b, x, 1.0)
    return None   # the general case is the pow primitive itself


def _huber_loss(b, op):
    if not _side_outputs_unused(op):
        return None
    x, label = op.operand_source(0), op.operand_source(1)
    d = float(_attr(op, "delta", default=1.0))
    r = sub(b, label, x)
    a = un(b, "pd_op.abs", r)
    small = sc(b, mul(b, r, r), 0.5)
    big = sc(b, a, d, -0.5 * d * d)
    return where(b, cmp(b, "pd_op.less_equal", a, scalar_like(b, a, d)), small, big)


def _one_hot(b, op):
    x = op.operand_source(0)
    n = _attr(op, "num_classes", "depth")
    if not _static(x) or n is None:
        return None
    n = int(n)
    classes = b.op2("pd_op.arange", [], [n], x.dtype, start=0, end=n, step=1, dtype=x.dtype)
    eq = cmp(b, "pd_op.equal", reshape(b, x, list(x.shape) + [1]), classes)
    return cast(b, eq, op.result(0).dtype or torch.float32)


def _squared_l2_norm(b, op):
    x = op.operand_source(0)
    if not _static(x):
        return None
    s = reduce(b, "pd_op.sum", mul(b, x, x), list(range(len(x.shape))), keepdim=False)
    return reshape(b, s, [1])


def _bce_loss(b, op):
    x, label = op.operand_source(0), op.operand_source(1)
    floor = scalar_like(b, x, -100.0)
    lx = b.op("pd_op.maximum", [un(b, "pd_op.log", x), floor], x)
    l1x = b.op("pd_op.maximum", [un(b, "pd_op.log", sc(b, x, -1.0, 1.0)), floor], x)
    return sc(b, add(b, mul(b, label, lx), mul(b, sc(b, label, -1.0, 1.0), l1x)), -1.0)


def _bmm(b, op):
    x, y = op.operand_source(0), op.operand_source(1)
    return b.op2("pd_op.matmul", [x, y], op.result(0).shape, x.dtype, transpose_x=False, transpose_y=False)


def _batch_norm(b, op):
    if not _side_outputs_unused(op):
        return None
    x = op.operand_source(0)
    if not _static(x):
        return None
    slots = op.attrs().get("__slots__")
    if slots:   # translated ProgramDesc op: operands by slot name
        ops = dict(zip(slots, op.operands()))
        mean, var, scale, bias = ops.get("Mean"), ops.get("Variance"), ops.get("Scale"), ops.get("Bias")
    else:       # PIR operand order: x, mean, variance, scale, bias
        o = op.operands() + [None] * 5
        mean, var, scale, bias = o[1], o[2], o[3], o[4]
    fmt = _attr(op, "data_format", "data_layout", default="NCHW")
    caxis = len(x.shape) - 1 if fmt in ("NHWC", "NLC", "NDHWC") else 1
    eps = float(_attr(op, "epsilon", default=1e-5))
    cshape = _channel_shape(x, caxis)
    use_global = bool(_attr(op, "is_test", default=False)) or bool(_attr(op, "use_global_stats", default=False))
    if use_global:
        if mean is None or var is None:
            return None
        m, v = reshape(b, mean, cshape), reshape(b, var, cshape)
        y = mul(b, sub(b, x, m), un(b, "pd_op.rsqrt", sc(b, v, 1.0, eps)))
    else:
        y, _, _ = _norm(b, x, [a for a in range(len(x.shape)) if a != caxis], eps)
    if scale is not None:
        y = mul(b, y, reshape(b, scale, cshape))
    if bias is not None:
        y = add(b, y, reshape(b, bias, cshape))
    return y


def _stack(b, op):
    xs = op.operands()
    if not xs or not all(_static(x) for x in xs):
        return None
    nd = len(xs[0].shape) + 1
    axis = int(_attr(op, "axis", default=0)) % nd
    parts = [reshape(b, x, list(x.shape[:axis]) + [1] + list(x.shape[axis:])) for x in xs]
    shape = list(xs[0].shape[:axis]) + [len(xs)] + list(xs[0].shape[axis:])
    return b.op2("pd_op.concat", parts, shape, xs[0].dtype, axis=axis)


def _unbind(b, op):
    """unbind / unstack along ``axis``: per index a unit slice reshaped without that axis (multi-output)."""
    x = op.operand_source(0)
    if not _static(x):
        return None
    nd = len(x.shape)
    axis = int(_attr(op, "axis", default=0)) % nd
    n = x.shape[axis]
    if n != op.num_results():
        return None
    out_shape = list(x.shape[:axis]) + list(x.shape[axis + 1:])
    outs = []
    for i in range(n):
        sl_shape = list(x.shape)
        sl_shape[axis] = 1
        sl = b.op2("pd_op.slice", [x], sl_shape, x.dtype, axis=axis, start=i, end=i + 1)
        outs.append(reshape(b, sl, out_shape))
    return outs


def _meshgrid(b, op):
    """meshgrid of k 1-D inputs (ij indexing): input i reshaped to size n_i on axis i and expanded to the grid."""
    xs = op.operands()
    if not xs or not all(_static(x) and len(x.shape) == 1 for x in xs) or op.num_results() != len(xs):
        return None
    grid = [x.shape[0] for x in xs]
    outs = []
    for i, x in enumerate(xs):
        shp = [1] * len(xs)
        shp[i] = grid[i]
        outs.append(b.op2("pd_op.expand", [reshape(b, x, shp)], grid, x.dtype, shape=grid))
    return outs


def _to_result_shape(b, op):
    """squeeze / unsqueeze / flatten: a reshape to the (static) result shape."""
    x, r = op.operand_source(0), op.result(0)
    if not _static(x) or r.shape is None or not _static(r) or not _side_outputs_unused(op):
        return None
    if _numel(x.shape) != _numel(r.shape):
        return None
    return reshape(b, x, r.shape)


def _add_n(b, op):
    xs = op.operands()
    if len(xs) < 2 or "axis" in op.attrs() or "dim" in op.attrs():
        return None   # pd_op.sum with one operand is the reduction, not add_n
    acc = xs[0]
    for x in xs[1:]:
        acc = add(b, acc, x)
    return acc


def _full_like(b, op):
    x = op.operand_source(0)
    if not _static(x):
        return None
    dt = _attr(op, "dtype", default=None)
    dt = dt if isinstance(dt, torch.dtype) else (op.result(0).dtype or x.dtype)
    return full(b, x.shape, float(_attr(op, "value", "fill_value", default=0.0)), dt)


def _dropout(b, op):
    if not _side_outputs_unused(op):
        return None
    x = op.operand_source(0)
    p = float(_attr(op, "p", "dropout_prob", default=0.5))
    mode = _attr(op, "mode", "dropout_implementation", default="upscale_in_train")
    if _attr(op, "is_test", default=False):
        return sc(b, x, 1.0) if mode == "upscale_in_train" else sc(b, x, 1.0 - p)
    if not _static(x):
        return None
    u = b.op2("pd_op.uniform", [], x.shape, torch.float32, shape=list(x.shape), min=0.0, max=1.0,
              seed=int(_attr(op, "seed", default=0)))
    keep = cast(b, cmp(b, "pd_op.greater_equal", u, full(b, x.shape, p, torch.float32)), x.dtype)
    y = mul(b, x, keep)
    return sc(b, y, 1.0 / (1.0 - p)) if mode == "upscale_in_train" and p < 1.0 else y


def _heaviside(b, op):
    x, y = op.operand_source(0), op.operand_source(1)
    pos = cast(b, cmp(b, "pd_op.greater_than", x, scalar_like(b, x, 0.0)), x.dtype)
    return where(b, cmp(b, "pd_op.equal", x, scalar_like(b, x, 0.0)), y, pos)


def _instance_norm(b, op):
    if not _side_outputs_unused(op):
        return None
    x = op.operand_source(0)
    if not _static(x) or len(x.shape) < 3:
        return None
    o = op.operands() + [None, None]
    scale, bias = o[1], o[2]
    y, _, _ = _norm(b, x, list(range(2, len(x.shape))), float(_attr(op, "epsilon", default=1e-5)))
    cs = _channel_shape(x, 1)
    if scale is not None:
        y = mul(b, y, reshape(b, scale, cs))
    if bias is not None:
        y = add(b, y, reshape(b, bias, cs))
    return y


def _clip(b, op):
    x = op.operand_source(0)
    if op.num_operands() != 1:
        return None
    lo = float(_attr(op, "min", default=-3.4e38))
    hi = float(_attr(op, "max", default=3.4e38))
    return b.op("pd_op.minimum", [b.op("pd_op.maximum", [x, scalar_like(b, x, lo)], x), scalar_like(b, x, hi)], x)


def _index_select(b, op):
    x, idx = op.operand_source(0), op.operand_source(1)
    axis = int(_attr(op, "axis", "dim", default=0)) % len(x.shape)
    return b.op2("pd_op.gather", [x, idx], op.result(0).shape, x.dtype, axis=axis)


def _group_norm(b, op):
    if not _side_outputs_unused(op):
        return None
    x = op.operand_source(0)
    if not _static(x) or _attr(op, "data_format", "data_layout", default="NCHW") != "NCHW":
        return None
    o = op.operands() + [None, None]
    scale, bias = o[1], o[2]
    g = int(_attr(op, "groups", default=1))
    N, C = x.shape[0], x.shape[1]
    xg = reshape(b, x, [N, g, _numel(x.shape[1:]) // g])
    y, _, _ = _norm(b, xg, [2], float(_attr(op, "epsilon", default=1e-5)))
    y = reshape(b, y, x.shape)
    cs = _channel_shape(x, 1)
    if scale is not None:
        y = mul(b, y, reshape(b, scale, cs))
    if bias is not None:
        y = add(b, y, reshape(b, bias, cs))
    return y


def _sigmoid_ce(b, op):
    if op.num_operands() != 2 or _attr(op, "normalize", default=False):
        return None
    x, label = op.operand_source(0), op.operand_source(1)
    zero = scalar_like(b, x, 0.0)
    nabs = sc(b, un(b, "pd_op.abs", x), -1.0)
    loss = add(b, sub(b, b.op("pd_op.maximum", [x, zero], x), mul(b, x, label)),
               un(b, "pd_op.log", sc(b, un(b, "pd_op.exp", nabs), 1.0, 1.0)))
    ig = _attr(op, "ignore_index", default=-100)
    keep = cmp(b, "pd_op.not_equal", label, scalar_like(b, label, float(ig)))
    return where(b, keep, loss, zero)


def _embedding(b, op):
    ids, w = op.operand_source(0), op.operand_source(1)
    if not _static(ids) or not _static(w):
        return None
    flat = reshape(b, ids, [_numel(ids.shape)])
    rows = b.op2("pd_op.gather", [w, flat], [_numel(ids.shape), w.shape[1]], w.dtype, axis=0)
    out = reshape(b, rows, list(ids.shape) + [w.shape[1]])
    pad = _attr(op, "padding_idx", default=-1)
    if pad is not None and int(pad) >= 0:
        hit = cmp(b, "pd_op.equal", reshape(b, ids, list(ids.shape) + [1]),
                  full(b, list(ids.shape) + [1], int(pad), ids.dtype))
        out = where(b, hit, full(b, out.shape, 0.0, w.dtype), out)
    return out


def _index_sample(b, op):
    x, idx = op.operand_source(0), op.operand_source(1)
    return b.op2("pd_op.take_along_axis", [x, idx], idx.shape, x.dtype, axis=1)


def _lerp(b, op):
    x, y, w = op.operand_source(0), op.operand_source(1), op.operand_source(2)
    return add(b, x, mul(b, w, sub(b, y, x)))


def _log_loss(b, op):
    x, label = op.operand_source(0), op.operand_source(1)
    eps = float(_attr(op, "epsilon", default=1e-4))
    a = mul(b, label, un(b, "pd_op.log", sc(b, x, 1.0, eps)))
    c = mul(b, sc(b, label, -1.0, 1.0), un(b, "pd_op.log", sc(b, x, -1.0, 1.0 + eps)))
    return sc(b, add(b, a, c), -1.0)


def _kldiv_loss(b, op):
    x, label = op.operand_source(0), op.operand_source(1)
    if not _static(x):
        return None
    if _attr(op, "log_target", default=False):
        loss = mul(b, un(b, "pd_op.exp", label), sub(b, label, x))
    else:
        out = mul(b, label, sub(b, un(b, "pd_op.log", label), x))
        loss = where(b, cmp(b, "pd_op.greater_than", label, scalar_like(b, label, 0.0)), out,
                     scalar_like(b, x, 0.0))
    red = _attr(op, "reduction", default="mean")
    allax = list(range(len(x.shape)))
    if red == "batchmean":
        s = reduce(b, "pd_op.sum", loss, allax, keepdim=False)
        return sc(b, s, 1.0 / x.shape[0]) if x.shape else s
    if red == "mean":
        return sc(b, reduce(b, "pd_op.sum", loss, allax, keepdim=False), 1.0 / max(1, _numel(x.shape)))
    if red == "sum":
        return reduce(b, "pd_op.sum", loss, allax, keepdim=False)
    return loss


def _softsign(b, op):
    x = op.operand_source(0)
    return div(b, x, sc(b, un(b, "pd_op.abs", x), 1.0, 1.0))


def _numel_rule(b, op):
    x = op.operand_source(0)
    if not _static(x):
        return None
    return full(b, [], _numel(x.shape), torch.int64)


# activations (python/paddle/decomposition/rules.py and the nn.functional definitions)
def _tanh_shrink(b, op):
    x = op.operand_source(0)
    return sub(b, x, un(b, "pd_op.tanh", x))


def _hardtanh(b, op):
    x = op.operand_source(0)
    lo, hi = float(_attr(op, "t_min", "min", default=-1.0)), float(_attr(op, "t_max", "max", default=1.0))
    return b.op("pd_op.minimum", [b.op("pd_op.maximum", [x, scalar_like(b, x, lo)], x), scalar_like(b, x, hi)], x)


def _selu(b, op):
    x = op.operand_source(0)
    s = float(_attr(op, "scale", default=1.0507009873554804934193349852946))
    a = float(_attr(op, "alpha", default=1.6732632423543772848170429916717))
    zero = scalar_like(b, x, 0.0)
    neg = sc(b, un(b, "pd_op.exp", b.op("pd_op.minimum", [x, zero], x)), a, -a)
    return sc(b, add(b, b.op("pd_op.maximum", [x, zero], x), neg), s)


def _celu(b, op):
    x = op.operand_source(0)
    a = float(_attr(op, "alpha", default=1.0))
    zero = scalar_like(b, x, 0.0)
    neg = sc(b, un(b, "pd_op.exp", sc(b, b.op("pd_op.minimum", [x, zero], x), 1.0 / a)), a, -a)
    return add(b, b.op("pd_op.maximum", [x, zero], x), neg)


def _thresholded_relu(b, op):
    x = op.operand_source(0)
    t = float(_attr(op, "threshold", default=1.0))
    return where(b, cmp(b, "pd_op.greater_than", x, scalar_like(b, x, t)), x, scalar_like(b, x, 0.0))


def _logsigmoid(b, op):
    # log(sigmoid(x)) = min(x, 0) - log(1 + exp(-|x|))
    x = op.operand_source(0)
    m = b.op("pd_op.minimum", [x, scalar_like(b, x, 0.0)], x)
    return sub(b, m, un(b, "pd_op.log", sc(b, un(b, "pd_op.exp", sc(b, un(b, "pd_op.abs", x), -1.0)), 1.0, 1.0)))


def _softshrink(b, op):
    x = op.operand_source(0)
    t = float(_attr(op, "threshold", "lambda", default=0.5))
    zero = scalar_like(b, x, 0.0)
    up = where(b, cmp(b, "pd_op.greater_than", x, scalar_like(b, x, t)), sc(b, x, 1.0, -t), zero)
    return where(b, cmp(b, "pd_op.less_than", x, scalar_like(b, x, -t)), sc(b, x, 1.0, t), up)


def _hardshrink(b, op):
    x = op.operand_source(0)
    t = float(_attr(op, "threshold", default=0.5))
    keep = cmp(b, "pd_op.greater_than", un(b, "pd_op.abs", x), scalar_like(b, x, t))
    return where(b, keep, x, scalar_like(b, x, 0.0))


def _log_base(base):
    def rule(b, op):
        x = op.operand_source(0)
        return sc(b, un(b, "pd_op.log", x), 1.0 / math.log(base))
    return rule


def _log1p(b, op):
    x = op.operand_source(0)
    return un(b, "pd_op.log", sc(b, x, 1.0, 1.0))


def _expm1(b, op):
    x = op.operand_source(0)
    return sc(b, un(b, "pd_op.exp", x), 1.0, -1.0)


def _stanh(b, op):
    x = op.operand_source(0)
    a, c = float(_attr(op, "scale_a", default=0.67)), float(_attr(op, "scale_b", default=1.7159))
    return sc(b, un(b, "pd_op.tanh", sc(b, x, a)), c)


RULES = {
    "pd_op.any": _any, "pd_op.mean_all": _mean_all, "pd_op.p_norm": _p_norm, "pd_op.pow": _pow,
    "pd_op.huber_loss": _huber_loss, "pd_op.one_hot": _one_hot, "pd_op.squared_l2_norm": _squared_l2_norm,
    "pd_op.bce_loss": _bce_loss, "pd_op.bmm": _bmm, "pd_op.batch_norm": _batch_norm, "pd_op.batch_norm_": _batch_norm,
    "pd_op.stack": _stack, "pd_op.unbind": _unbind, "pd_op.unstack": _unbind, "pd_op.meshgrid": _meshgrid,
    "pd_op.squeeze": _to_result_shape, "pd_op.unsqueeze": _to_result_shape,
    "pd_op.squeeze2": _to_result_shape, "pd_op.unsqueeze2": _to_result_shape, "pd_op.flatten": _to_result_shape,
    "pd_op.add_n": _add_n, "pd_op.sum": _add_n, "pd_op.full_like": _full_like, "pd_op.dropout": _dropout, "pd_op.heaviside": _heaviside,
    "pd_op.instance_norm": _instance_norm, "pd_op.clip": _clip, "pd_op.index_select": _index_select,
    "pd_op.group_norm": _group_norm, "pd_op.sigmoid_cross_entropy_with_logits": _sigmoid_ce,
    "pd_op.embedding": _embedding, "pd_op.index_sample": _index_sample, "pd_op.lerp": _lerp,
    "pd_op.log_loss": _log_loss, "pd_op.kldiv_loss": _kldiv_loss, "pd_op.softsign": _softsign,
    "pd_op.numel": _numel_rule, "pd_op.tanh_shrink": _tanh_shrink, "pd_op.hardtanh": _hardtanh,
    "pd_op.brelu": _hardtanh, "pd_op.selu": _selu, "pd_op.celu": _celu, "pd_op.thresholded_relu": _thresholded_relu,
    "pd_op.logsigmoid": _logsigmoid, "pd_op.softshrink": _softshrink, "pd_op.hardshrink": _hardshrink,
    "pd_op.log2": _log_base(2.0), "pd_op.log10": _log_base(10.0), "pd_op.log1p": _log1p, "pd_op.expm1": _expm1,
    "pd_op.stanh": _stanh,
}
