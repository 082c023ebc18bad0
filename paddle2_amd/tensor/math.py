"""Math ops (reference: python/paddle/tensor/math.py, ops.py).

Elementwise long-tail ops run on ATen-on-ROCm (SURVEY §7.1 "long tail binds to ATen");
the LLM hot ops live in :mod:`paddle2_amd.ops` as hand-written HIP kernels.
"""
from __future__ import annotations

import torch

from ..framework import dtype as _dt
from ..framework.tensor import Tensor
from ._helpers import axis_arg, dtype_arg, scalar, u, ut, w
from ..amp import amp_op as _amp_op  # noqa: E402

_wrap = Tensor._wrap


def _unary(fn, name):
    def op(x, name=None):
        return _wrap(fn(x._t if isinstance(x, Tensor) else ut(x)))

    op.__name__ = name
    op.__doc__ = f"paddle.{name} (elementwise, ATen on ROCm)."
    return op


def _unary_inplace(fn_, name):
    def op(x, name=None):
        fn_(x._t)
        return x

    op.__name__ = name
    return op


_UNARY = {
    "abs": torch.abs, "acos": torch.acos, "acosh": torch.acosh, "asin": torch.asin, "asinh": torch.asinh,
    "atan": torch.atan, "atanh": torch.atanh, "ceil": torch.ceil, "cos": torch.cos, "cosh": torch.cosh,
    "exp": torch.exp, "expm1": torch.expm1, "floor": torch.floor, "log": torch.log, "log2": torch.log2,
    "log10": torch.log10, "log1p": torch.log1p, "reciprocal": torch.reciprocal, "rsqrt": torch.rsqrt,
    "sin": torch.sin, "sinh": torch.sinh, "sqrt": torch.sqrt, "square": torch.square, "tan": torch.tan,
    "tanh": torch.tanh, "sign": torch.sign, "sgn": torch.sgn, "erf": torch.erf, "erfinv": torch.erfinv,
    "trunc": torch.trunc, "frac": torch.frac, "lgamma": torch.lgamma, "digamma": torch.digamma,
    "neg": torch.neg, "i0": torch.i0, "i0e": torch.special.i0e, "i1": torch.special.i1,
    "i1e": torch.special.i1e, "deg2rad": torch.deg2rad, "rad2deg": torch.rad2deg, "angle": torch.angle,
    "conj": torch.conj_physical, "real": torch.real, "imag": torch.imag, "sigmoid": torch.sigmoid,
    "isnan": torch.isnan, "isinf": torch.isinf, "isfinite": torch.isfinite, "isposinf": torch.isposinf,
    "isneginf": torch.isneginf, "isreal": torch.isreal, "signbit": torch.signbit, "exp2": torch.exp2,
    "gammaln": torch.lgamma, "sinc": torch.sinc, "positive": torch.positive,
    "bitwise_not": torch.bitwise_not, "logical_not": torch.logical_not,
}

for _n, _f in _UNARY.items():
    globals()[_n] = _unary(_f, _n)

_INPLACE = {
    "abs_": torch.Tensor.abs_, "ceil_": torch.Tensor.ceil_, "cos_": torch.Tensor.cos_, "exp_": torch.Tensor.exp_,
    "floor_": torch.Tensor.floor_, "log_": torch.Tensor.log_, "reciprocal_": torch.Tensor.reciprocal_,
    "rsqrt_": torch.Tensor.rsqrt_, "sin_": torch.Tensor.sin_, "sqrt_": torch.Tensor.sqrt_,
    "square_": torch.Tensor.square_, "tanh_": torch.Tensor.tanh_, "trunc_": torch.Tensor.trunc_,
    "sigmoid_": torch.Tensor.sigmoid_, "neg_": torch.Tensor.neg_, "erf_": torch.Tensor.erf_,
    "sign_": torch.Tensor.sign_, "tan_": torch.Tensor.tan_, "log1p_": torch.Tensor.log1p_,
    "expm1_": torch.Tensor.expm1_, "frac_": torch.Tensor.frac_, "digamma_": torch.Tensor.digamma_,
    "lgamma_": torch.Tensor.lgamma_, "acos_": torch.Tensor.acos_, "asin_": torch.Tensor.asin_,
    "atan_": torch.Tensor.atan_, "cosh_": torch.Tensor.cosh_, "sinh_": torch.Tensor.sinh_,
    "log2_": torch.Tensor.log2_, "log10_": torch.Tensor.log10_, "i0_": torch.Tensor.i0_,
}
for _n, _f in _INPLACE.items():
    globals()[_n] = _unary_inplace(_f, _n)


def round(x, decimals=0, name=None):
    return _wrap(torch.round(x._t, decimals=decimals))


def round_(x, decimals=0, name=None):
    x._t.round_(decimals=decimals)
    return x


# ------------------------------------------------------------------ binary
def _bin(a, b):
    if isinstance(a, Tensor):
        ta = a._t
        tb = b._t if isinstance(b, Tensor) else (b if not hasattr(b, "__len__") else ut(b, ta))
        return ta, tb
    tb = ut(b)
    return ut(a, tb), tb


def add(x, y, name=None):
    a, b = _bin(x, y)
    return _wrap(a + b)


def subtract(x, y, name=None):
    a, b = _bin(x, y)
    return _wrap(a - b)


def multiply(x, y, name=None):
    a, b = _bin(x, y)
    return _wrap(a * b)


def divide(x, y, name=None):
    a, b = _bin(x, y)
    if isinstance(a, torch.Tensor) and not a.is_floating_point() and not a.is_complex() and \
            (not isinstance(b, torch.Tensor) or not b.is_floating_point()) and not isinstance(b, float):
        # paddle: int / int -> float32 true division
        return _wrap(torch.true_divide(a, b).to(_dt.default_float_dtype()))
    return _wrap(a / b)


def floor_divide(x, y, name=None):
    a, b = _bin(x, y)
    return _wrap(torch.floor_divide(a, b))


def remainder(x, y, name=None):
    a, b = _bin(x, y)
    return _wrap(torch.remainder(a, b))


mod = remainder
floor_mod = remainder


def pow(x, y, name=None):
    a, b = _bin(x, y)
    return _wrap(torch.pow(a, b))


def float_power(x, y, name=None):
    a, b = _bin(x, y)
    return _wrap(torch.float_power(a, b))


def maximum(x, y, name=None):
    a, b = _bin(x, y)
    return _wrap(torch.maximum(a, ut(b, a)))


def minimum(x, y, name=None):
    a, b = _bin(x, y)
    return _wrap(torch.minimum(a, ut(b, a)))


def fmax(x, y, name=None):
    return _wrap(torch.fmax(ut(x), ut(y)))


def fmin(x, y, name=None):
    return _wrap(torch.fmin(ut(x), ut(y)))


def atan2(x, y, name=None):
    return _wrap(torch.atan2(ut(x), ut(y)))


def hypot(x, y, name=None):
    return _wrap(torch.hypot(ut(x), ut(y)))


def copysign(x, y, name=None):
    return _wrap(torch.copysign(ut(x), ut(y)))


def nextafter(x, y, name=None):
    return _wrap(torch.nextafter(ut(x), ut(y)))


def ldexp(x, y, name=None):
    return _wrap(torch.ldexp(ut(x), ut(y)))


def heaviside(x, y, name=None):
    return _wrap(torch.heaviside(ut(x), ut(y)))


def gcd(x, y, name=None):
    return _wrap(torch.gcd(ut(x), ut(y)))


def lcm(x, y, name=None):
    return _wrap(torch.lcm(ut(x), ut(y)))


def logaddexp(x, y, name=None):
    return _wrap(torch.logaddexp(ut(x), ut(y)))


def bitwise_and(x, y, out=None, name=None):
    return _wrap(torch.bitwise_and(ut(x), ut(y)))


def bitwise_or(x, y, out=None, name=None):
    return _wrap(torch.bitwise_or(ut(x), ut(y)))


def bitwise_xor(x, y, out=None, name=None):
    return _wrap(torch.bitwise_xor(ut(x), ut(y)))


def bitwise_left_shift(x, y, is_arithmetic=True, out=None, name=None):
    return _wrap(torch.bitwise_left_shift(ut(x), ut(y)))


def bitwise_right_shift(x, y, is_arithmetic=True, out=None, name=None):
    return _wrap(torch.bitwise_right_shift(ut(x), ut(y)))


def _inplace_bin(fn):
    def op(x, y, name=None):
        b = y._t if isinstance(y, Tensor) else y
        fn(x._t, b)
        return x

    return op


add_ = _inplace_bin(torch.Tensor.add_)
subtract_ = _inplace_bin(torch.Tensor.sub_)
multiply_ = _inplace_bin(torch.Tensor.mul_)
divide_ = _inplace_bin(torch.Tensor.div_)
pow_ = _inplace_bin(torch.Tensor.pow_)
remainder_ = _inplace_bin(torch.Tensor.remainder_)
mod_ = remainder_
floor_divide_ = _inplace_bin(torch.Tensor.floor_divide_)


def scale(x, scale=1.0, bias=0.0, bias_after_scale=True, act=None, name=None):
    """paddle.scale: out = scale*x + bias (or scale*(x+bias))."""
    s = scalar(scale)
    t = x._t
    out = t * s + bias if bias_after_scale else (t + bias) * s
    if act is not None:
        out = getattr(torch, act)(out)
    return _wrap(out.to(t.dtype) if out.dtype != t.dtype and t.is_floating_point() else out)


def scale_(x, scale=1.0, bias=0.0, bias_after_scale=True, act=None, name=None):
    s = scalar(scale)
    if bias_after_scale:
        x._t.mul_(s).add_(bias)
    else:
        x._t.add_(bias).mul_(s)
    return x


def stanh(x, scale_a=0.67, scale_b=1.7159, name=None):
    return _wrap(scale_b * torch.tanh(scale_a * x._t))


def clip(x, min=None, max=None, name=None):
    lo = scalar(min) if not (isinstance(min, Tensor) and min.size > 1) else min._t
    hi = scalar(max) if not (isinstance(max, Tensor) and max.size > 1) else max._t
    t = x._t
    if not t.is_floating_point() and (isinstance(lo, float) or isinstance(hi, float)):
        lo = None if lo is None else int(lo)
        hi = None if hi is None else int(hi)
    return _wrap(torch.clamp(t, lo, hi))


def clip_(x, min=None, max=None, name=None):
    x._t.clamp_(scalar(min), scalar(max))
    return x


def lerp(x, y, weight, name=None):
    wt = weight._t if isinstance(weight, Tensor) else weight
    return _wrap(torch.lerp(x._t, ut(y, x._t), wt))


def lerp_(x, y, weight, name=None):
    x._t.lerp_(ut(y, x._t), weight._t if isinstance(weight, Tensor) else weight)
    return x


def logit(x, eps=None, name=None):
    return _wrap(torch.logit(x._t, eps))


def nan_to_num(x, nan=0.0, posinf=None, neginf=None, name=None):
    return _wrap(torch.nan_to_num(x._t, nan, posinf, neginf))


def increment(x, value=1.0, name=None):
    with torch.no_grad():
        x._t.add_(value)
    return x


# ------------------------------------------------------------- reductions
def _sum_dtype(t, dtype):
    if dtype is not None:
        return _dt.convert_dtype(dtype)
    if t.dtype in (torch.bool, torch.int32, torch.int16, torch.int8, torch.uint8):
        return torch.int64
    return None


@_amp_op("sum")
def sum(x, axis=None, dtype=None, keepdim=False, name=None):
    t = x._t if isinstance(x, Tensor) else ut(x)
    ax = axis_arg(axis)
    dt = _sum_dtype(t, dtype)
    if ax is None:
        r = torch.sum(t, dtype=dt)
        if keepdim:
            r = r.reshape([1] * t.dim())
        return _wrap(r)
    return _wrap(torch.sum(t, dim=ax, keepdim=keepdim, dtype=dt))


def nansum(x, axis=None, dtype=None, keepdim=False, name=None):
    ax = axis_arg(axis)
    return _wrap(torch.nansum(x._t, dim=ax, keepdim=keepdim, dtype=dtype_arg(dtype)))


@_amp_op("mean")
def mean(x, axis=None, keepdim=False, name=None):
    t = x._t
    ax = axis_arg(axis)
    if ax is None:
        r = torch.mean(t)
        return _wrap(r.reshape([1] * t.dim()) if keepdim else r)
    return _wrap(torch.mean(t, dim=ax, keepdim=keepdim))


def nanmean(x, axis=None, keepdim=False, name=None):
    return _wrap(torch.nanmean(x._t, dim=axis_arg(axis), keepdim=keepdim))


def prod(x, axis=None, keepdim=False, dtype=None, name=None):
    t = x._t
    ax = axis_arg(axis)
    dt = dtype_arg(dtype)
    if ax is None:
        r = torch.prod(t, dtype=dt)
        return _wrap(r.reshape([1] * t.dim()) if keepdim else r)
    if isinstance(ax, tuple):
        r = t if dt is None else t.to(dt)
        for a in sorted((a % t.dim() for a in ax), reverse=True):
            r = torch.prod(r, dim=a, keepdim=keepdim)
        return _wrap(r)
    return _wrap(torch.prod(t, dim=ax, keepdim=keepdim, dtype=dt))


def _minmax(fn_all, fn_dim):
    def op(x, axis=None, keepdim=False, name=None):
        t = x._t
        ax = axis_arg(axis)
        if ax is None:
            r = fn_all(t)
            return _wrap(r.reshape([1] * t.dim()) if keepdim else r)
        return _wrap(fn_dim(t, dim=ax, keepdim=keepdim))

    return op


max = _minmax(torch.amax, torch.amax)
min = _minmax(torch.amin, torch.amin)
amax = max
amin = min


def logsumexp(x, axis=None, keepdim=False, name=None):
    t = x._t
    ax = axis_arg(axis)
    if ax is None:
        ax = tuple(range(t.dim()))
    return _wrap(torch.logsumexp(t, dim=ax, keepdim=keepdim))


def cumsum(x, axis=None, dtype=None, name=None):
    t = x._t
    if axis is None:
        t = t.flatten()
        axis = 0
    return _wrap(torch.cumsum(t, dim=int(axis), dtype=dtype_arg(dtype)))


def cumsum_(x, axis=None, dtype=None, name=None):
    x._t.cumsum_(dim=0 if axis is None else int(axis))
    return x


def cumprod(x, dim=None, dtype=None, name=None):
    t = x._t
    if dim is None:
        t = t.flatten()
        dim = 0
    return _wrap(torch.cumprod(t, dim=int(dim), dtype=dtype_arg(dtype)))


def cummax(x, axis=None, dtype="int64", name=None):
    t = x._t
    if axis is None:
        t, axis = t.flatten(), 0
    v, i = torch.cummax(t, int(axis))
    return _wrap(v), _wrap(i.to(_dt.convert_dtype(dtype)))


def cummin(x, axis=None, dtype="int64", name=None):
    t = x._t
    if axis is None:
        t, axis = t.flatten(), 0
    v, i = torch.cummin(t, int(axis))
    return _wrap(v), _wrap(i.to(_dt.convert_dtype(dtype)))


def logcumsumexp(x, axis=None, dtype=None, name=None):
    t = x._t
    if axis is None:
        t, axis = t.flatten(), 0
    return _wrap(torch.logcumsumexp(t if dtype is None else t.to(dtype_arg(dtype)), int(axis)))


def all(x, axis=None, keepdim=False, name=None):
    t = x._t
    ax = axis_arg(axis)
    if ax is None:
        r = torch.all(t)
        return _wrap(r.reshape([1] * t.dim()) if keepdim else r)
    return _wrap(torch.all(t, dim=ax, keepdim=keepdim))


def any(x, axis=None, keepdim=False, name=None):
    t = x._t
    ax = axis_arg(axis)
    if ax is None:
        r = torch.any(t)
        return _wrap(r.reshape([1] * t.dim()) if keepdim else r)
    return _wrap(torch.any(t, dim=ax, keepdim=keepdim))


def count_nonzero(x, axis=None, keepdim=False, name=None):
    t = x._t
    ax = axis_arg(axis)
    r = torch.count_nonzero(t, dim=ax)
    if keepdim:
        if ax is None:
            r = r.reshape([1] * t.dim())
        else:
            for a in sorted([ax] if isinstance(ax, int) else list(ax)):
                r = r.unsqueeze(a % t.dim())
    return _wrap(r)


def diff(x, n=1, axis=-1, prepend=None, append=None, name=None):
    return _wrap(torch.diff(x._t, n=n, dim=axis, prepend=None if prepend is None else ut(prepend),
                            append=None if append is None else ut(append)))


def trace(x, offset=0, axis1=0, axis2=1, name=None):
    return _wrap(torch.diagonal(x._t, offset, axis1, axis2).sum(-1))


def diagonal(x, offset=0, axis1=0, axis2=1, name=None):
    return _wrap(torch.diagonal(x._t, offset, axis1, axis2))


def kron(x, y, name=None):
    return _wrap(torch.kron(ut(x), ut(y)))


def inner(x, y, name=None):
    return _wrap(torch.inner(ut(x), ut(y)))


def outer(x, y, name=None):
    return _wrap(torch.outer(ut(x).flatten(), ut(y).flatten()))


def multiplex(inputs, index, name=None):
    stacked = torch.stack([i._t for i in inputs], 0)
    idx = index._t.flatten().long()
    return _wrap(stacked[idx, torch.arange(idx.numel(), device=idx.device)])


def add_n(inputs, name=None):
    if isinstance(inputs, Tensor):
        return inputs
    r = inputs[0]._t
    for t in inputs[1:]:
        r = r + t._t
    return _wrap(r)


def renorm(x, p, axis, max_norm):
    return _wrap(torch.renorm(x._t, p, axis, max_norm))


def cartesian_prod(x, name=None):
    return _wrap(torch.cartesian_prod(*[t._t for t in x]))


def take(x, index, mode="raise", name=None):
    t = x._t.flatten()
    idx = index._t.long()
    n = t.numel()
    if mode == "wrap":
        idx = idx % n
    elif mode == "clip":
        idx = idx.clamp(0, n - 1)
    else:
        idx = torch.where(idx < 0, idx + n, idx)
    return _wrap(t[idx])


def polygamma(x, n, name=None):
    return _wrap(torch.polygamma(n, x._t))


def multigammaln(x, p, name=None):
    return _wrap(torch.mvlgamma(x._t, p))


def log_normal_(x, mean=1.0, std=2.0, name=None):
    with torch.no_grad():
        x._t.log_normal_(mean, std)
    return x


def combinations(x, r=2, with_replacement=False, name=None):
    return _wrap(torch.combinations(x._t, r, with_replacement))


def signbit_(x):
    return signbit(x)  # noqa: F821


def addmm(input, x, y, beta=1.0, alpha=1.0, name=None):
    return _wrap(torch.addmm(input._t, x._t, y._t, beta=beta, alpha=alpha))


def baddbmm(input, x, y, beta=1.0, alpha=1.0, name=None):
    return _wrap(torch.baddbmm(input._t, x._t, y._t, beta=beta, alpha=alpha))


def isin(x, test_x, assume_unique=False, invert=False, name=None):
    return _wrap(torch.isin(x._t, test_x._t, assume_unique=assume_unique, invert=invert))


def trapezoid(y, x=None, dx=None, axis=-1, name=None):
    if x is not None:
        return _wrap(torch.trapezoid(y._t, x._t, dim=axis))
    return _wrap(torch.trapezoid(y._t, dx=1.0 if dx is None else dx, dim=axis))


def cumulative_trapezoid(y, x=None, dx=None, axis=-1, name=None):
    if x is not None:
        return _wrap(torch.cumulative_trapezoid(y._t, x._t, dim=axis))
    return _wrap(torch.cumulative_trapezoid(y._t, dx=1.0 if dx is None else dx, dim=axis))


__all__ = [_n for _n, _v in list(globals().items())
           if not _n.startswith("_") and callable(_v) and getattr(_v, "__module__", None) == __name__]
