"""Remaining ``paddle.*`` names of the reference ``__all__`` (python/paddle/__init__.py): the in-place ``op_``
twins of existing ops, plus block_diag / dsplit / frexp / gammainc(c) / histogram_bin_edges / histogramdd /
log_normal / pdist / reduce_as / reverse and ``LazyGuard`` (reference python/paddle/tensor/{math,linalg,
manipulation,random}.py, python/paddle/nn/initializer/lazy_init.py).

An in-place twin computes the out-of-place op and writes the result into ``x`` (cast to x's dtype, as the
reference's inplace kernels do for comparison / logical ops) and returns ``x``; the result must have x's
shape.  Autograd sees one in-place copy, so a leaf that requires grad is rejected exactly like torch does.
"""
from __future__ import annotations

import torch

from ..framework.tensor import Tensor
from . import creation as _c
from . import logic as _lg
from . import manipulation as _mp
from . import math as _mt
from ._helpers import ut

_wrap = Tensor._wrap

__all__ = ["block_diag", "dsplit", "frexp", "gammainc", "gammaincc", "histogram_bin_edges", "histogramdd",
           "log_normal", "pdist", "reduce_as", "reverse", "LazyGuard"]


def _inplace_of(fn, name):
    def op(x, *args, **kwargs):
        out = ut(fn(x, *args, **kwargs))
        if tuple(out.shape) != tuple(x._t.shape):
            raise ValueError(f"{name}: the result shape {list(out.shape)} cannot be written into x of shape "
                             f"{list(x._t.shape)} in place")
        x._t.copy_(out)
        return x

    op.__name__ = op.__qualname__ = name
    op.__doc__ = f"In-place version of ``{fn.__name__}`` (writes into ``x`` and returns it)."
    return op


_INPLACE = {
    "addmm_": _mt.addmm, "cumprod_": _mt.cumprod, "logit_": _mt.logit, "floor_mod_": _mt.floor_mod,
    "bitwise_and_": _mt.bitwise_and, "bitwise_or_": _mt.bitwise_or, "bitwise_xor_": _mt.bitwise_xor,
    "bitwise_not_": _mt.bitwise_not, "bitwise_left_shift_": _mt.bitwise_left_shift,
    "bitwise_right_shift_": _mt.bitwise_right_shift, "gcd_": _mt.gcd, "lcm_": _mt.lcm, "renorm_": _mt.renorm,
    "multigammaln_": _mt.multigammaln, "nan_to_num_": _mt.nan_to_num, "ldexp_": _mt.ldexp,
    "polygamma_": _mt.polygamma, "copysign_": _mt.copysign, "hypot_": _mt.hypot, "sinc_": _mt.sinc,
    "gammaln_": _mt.gammaln, "equal_": _lg.equal, "less_than_": _lg.less_than, "less_equal_": _lg.less_equal,
    "greater_than_": _lg.greater_than, "greater_equal_": _lg.greater_equal, "logical_and_": _lg.logical_and,
    "logical_or_": _lg.logical_or, "logical_not_": _mt.logical_not, "triu_": _c.triu, "tril_": _c.tril,
    "index_fill_": _mp.index_fill, "masked_scatter_": _mp.masked_scatter,
}


def gammainc(x, y, name=None):
    """Regularized lower incomplete gamma P(x, y) (reference math.py gammainc)."""
    return _wrap(torch.special.gammainc(ut(x), ut(y)))


def gammaincc(x, y, name=None):
    """Regularized upper incomplete gamma Q(x, y) = 1 - P(x, y)."""
    return _wrap(torch.special.gammaincc(ut(x), ut(y)))


_INPLACE["gammainc_"] = gammainc
_INPLACE["gammaincc_"] = gammaincc

for _n, _f in _INPLACE.items():
    globals()[_n] = _inplace_of(_f, _n)
    __all__.append(_n)


def t_(input, name=None):
    """In-place transpose of a 0/1/2-D tensor (reference math.py t_)."""
    if input._t.dim() > 2:
        raise ValueError(f"t_ expects a tensor of at most 2 dims, got {input._t.dim()}")
    input._t.t_()
    return input


__all__.append("t_")


def block_diag(inputs, name=None):
    return _wrap(torch.block_diag(*[ut(x) for x in inputs]))


def dsplit(x, num_or_indices, name=None):
    """Split along axis 2 (x needs >= 3 dims), like numpy.dsplit."""
    if ut(x).dim() < 3:
        raise ValueError("dsplit expects a tensor with at least 3 dims")
    return [_wrap(t) for t in torch.tensor_split(ut(x), num_or_indices, dim=2)] if isinstance(
        num_or_indices, (list, tuple)) else [_wrap(t) for t in torch.tensor_split(ut(x), int(num_or_indices), dim=2)]


def frexp(x, name=None):
    """(mantissa, exponent) with x = mantissa * 2**exponent, |mantissa| in [0.5, 1); both in x's dtype."""
    t = ut(x)
    if t.dtype not in (torch.float32, torch.float64):
        raise TypeError(f"frexp: the data type of input must be float32 or float64, got {t.dtype}")
    m, e = torch.frexp(t)
    return _wrap(m), _wrap(e.to(t.dtype))


def histogram_bin_edges(input, bins=100, min=0, max=0, name=None):
    t = ut(input)
    if max == 0 and min == 0:
        lo, hi = float(t.min()), float(t.max())
    else:
        if max < min:
            raise ValueError("max must be larger than min in range parameter")
        lo, hi = float(min), float(max)
    if hi == lo:
        lo, hi = lo - 0.5, hi + 0.5
    dt = t.dtype if t.is_floating_point() else torch.float32
    return _wrap(torch.linspace(lo, hi, int(bins) + 1, dtype=dt, device=t.device))


def histogramdd(x, bins=10, ranges=None, density=False, weights=None, name=None):
    """-> (hist, [bin edges per dim]) of the rows of x [N, D] (computed on the host, returned on x's device)."""
    t = ut(x)
    w = ut(weights).cpu() if weights is not None else None
    rng = None if ranges is None else [float(r) for r in ranges]
    b = bins if isinstance(bins, int) else [ut(e).cpu() if not isinstance(e, int) else e for e in bins]
    h, edges = torch.histogramdd(t.detach().cpu(), bins=b, range=rng, weight=w, density=density)
    return _wrap(h.to(t.device)), [_wrap(e.to(t.device)) for e in edges]


def log_normal(mean=1.0, std=2.0, shape=None, dtype=None, name=None):
    """Samples exp(N(mean, std^2)) (reference random.py log_normal)."""
    from ..framework.dtype import convert_dtype, get_default_dtype
    from ..framework.place import current_torch_device

    dt = convert_dtype(dtype) if dtype is not None else convert_dtype(get_default_dtype())
    dev = current_torch_device()
    if isinstance(mean, Tensor) or isinstance(std, Tensor):
        mu, sd = ut(mean) if isinstance(mean, Tensor) else mean, ut(std) if isinstance(std, Tensor) else std
        mu_t = mu if isinstance(mu, torch.Tensor) else torch.full_like(sd, float(mu))
        sd_t = sd if isinstance(sd, torch.Tensor) else torch.full_like(mu_t, float(sd))
        return _wrap(torch.exp(torch.normal(mu_t, sd_t)).to(dt))
    shp = [int(s) for s in (ut(shape).tolist() if isinstance(shape, Tensor) else (shape or [1]))]
    return _wrap(torch.empty(shp, dtype=dt, device=dev).log_normal_(float(mean), float(std)))


def pdist(x, p=2.0, name=None):
    """Condensed pairwise p-norm distances between the rows of x [N, M] -> [N*(N-1)/2]."""
    return _wrap(torch.nn.functional.pdist(ut(x), p=p))


def reduce_as(x, target, name=None):
    """Sum x over the broadcast dimensions so the result has target's shape (reference math.py reduce_as)."""
    t, shp = ut(x), list(ut(target).shape)
    lead = t.dim() - len(shp)
    if lead < 0:
        raise ValueError("reduce_as: target has more dims than x")
    out = t.sum(dim=list(range(lead))) if lead else t
    dims = [i for i, (a, b) in enumerate(zip(out.shape, shp)) if b == 1 and a != 1]
    if dims:
        out = out.sum(dim=dims, keepdim=True)
    if list(out.shape) != shp:
        raise ValueError(f"reduce_as: cannot reduce {list(t.shape)} to {shp}")
    return _wrap(out)


def reverse(x, axis, name=None):
    """Flip along ``axis`` (int or list) — the legacy fluid reverse op."""
    axes = [axis] if isinstance(axis, int) else list(axis)
    return _wrap(torch.flip(ut(x), axes))


class LazyGuard:
    """paddle.LazyGuard (nn/initializer/lazy_init.py): parameters created inside are initialised lazily in the
    reference.  Here parameter storage is created on the device at construction (288 GB HBM per MI355X holds
    every config we run), so the guard only records that it was entered; ``Layer`` initialisation is
    unchanged and ``startup_program`` has nothing to replay."""

    active = False

    def __enter__(self):
        self._prev = LazyGuard.active
        LazyGuard.active = True
        return self

    def __exit__(self, *exc):
        LazyGuard.active = self._prev
        return False

