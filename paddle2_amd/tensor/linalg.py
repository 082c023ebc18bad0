"""Linear algebra (reference: python/paddle/tensor/linalg.py).

``matmul`` is the plain library GEMM (hipBLASLt via ATen on ROCm, reference path
funcs/blas/blaslt_impl.hip.h); fused GEMM epilogues live in :mod:`paddle2_amd.ops`.
"""
from __future__ import annotations

import torch

from ..framework.tensor import Tensor
from ._helpers import axis_arg, ut
from ..amp import amp_op as _amp_op  # noqa: E402

_wrap = Tensor._wrap


@_amp_op("matmul")
def matmul(x, y, transpose_x=False, transpose_y=False, name=None):
    a = x._t
    b = y._t
    if transpose_x:
        a = a.transpose(-1, -2) if a.dim() > 1 else a
    if transpose_y:
        b = b.transpose(-1, -2) if b.dim() > 1 else b
    return _wrap(torch.matmul(a, b))


def mm(input, mat2, name=None):
    return _wrap(torch.matmul(input._t, mat2._t))


def bmm(x, y, name=None):
    return _wrap(torch.bmm(x._t, y._t))


def mv(x, vec, name=None):
    return _wrap(torch.mv(x._t, vec._t))


def dot(x, y, name=None):
    a, b = x._t, y._t
    if a.dim() == 2:
        return _wrap((a * b).sum(-1))
    return _wrap(torch.dot(a, b))


def vecdot(x, y, axis=-1, name=None):
    return _wrap(torch.linalg.vecdot(x._t, y._t, dim=axis))


def einsum(equation, *operands):
    if len(operands) == 1 and isinstance(operands[0], (list, tuple)):
        operands = operands[0]
    return _wrap(torch.einsum(equation, *[o._t for o in operands]))


def tensordot(x, y, axes=2, name=None):
    if isinstance(axes, Tensor):
        axes = axes._t.tolist()
    return _wrap(torch.tensordot(x._t, y._t, dims=axes))


def multi_dot(x, name=None):
    return _wrap(torch.linalg.multi_dot([t._t for t in x]))


def norm(x, p=None, axis=None, keepdim=False, name=None):
    t = x._t
    ax = axis_arg(axis)
    if p is None or p == "fro":
        if ax is None:
            return _wrap(torch.linalg.vector_norm(t.flatten(), 2).reshape([1] * t.dim()) if keepdim
                         else torch.linalg.vector_norm(t.flatten(), 2))
        if isinstance(ax, tuple) and len(ax) == 2 and p == "fro":
            return _wrap(torch.linalg.matrix_norm(t, "fro", dim=ax, keepdim=keepdim))
        return _wrap(torch.linalg.vector_norm(t, 2, dim=ax, keepdim=keepdim))
    if p == "nuc":
        return _wrap(torch.linalg.matrix_norm(t, "nuc", dim=ax or (-2, -1), keepdim=keepdim))
    if isinstance(ax, tuple) and len(ax) == 2 and p in (1, -1, 2, -2, float("inf"), float("-inf")):
        return _wrap(torch.linalg.matrix_norm(t, p, dim=ax, keepdim=keepdim))
    if ax is None:
        t = t.flatten()
        r = torch.linalg.vector_norm(t, p)
        return _wrap(r.reshape([1] * x._t.dim()) if keepdim else r)
    return _wrap(torch.linalg.vector_norm(t, p, dim=ax, keepdim=keepdim))


def vector_norm(x, p=2.0, axis=None, keepdim=False, name=None):
    return _wrap(torch.linalg.vector_norm(x._t, p, dim=axis_arg(axis), keepdim=keepdim))


def matrix_norm(x, p="fro", axis=[-2, -1], keepdim=False, name=None):
    return _wrap(torch.linalg.matrix_norm(x._t, p, dim=tuple(axis), keepdim=keepdim))


def dist(x, y, p=2, name=None):
    return _wrap(torch.dist(x._t, y._t, p))


def cross(x, y, axis=9, name=None):
    a, b = x._t, y._t
    if axis == 9:
        axis = next(i for i, s in enumerate(a.shape) if s == 3)
    return _wrap(torch.linalg.cross(a, b, dim=axis))


def cholesky(x, upper=False, name=None):
    return _wrap(torch.linalg.cholesky(x._t, upper=upper))


def cholesky_solve(x, y, upper=False, name=None):
    return _wrap(torch.cholesky_solve(x._t, y._t, upper=upper))


def cholesky_inverse(x, upper=False, name=None):
    return _wrap(torch.cholesky_inverse(x._t, upper=upper))


def matrix_power(x, n, name=None):
    return _wrap(torch.linalg.matrix_power(x._t, n))


def det(x, name=None):
    return _wrap(torch.linalg.det(x._t))


def slogdet(x, name=None):
    s, l = torch.linalg.slogdet(x._t)
    return _wrap(torch.stack([s, l]))


def inverse(x, name=None):
    return _wrap(torch.linalg.inv(x._t))


inv = inverse


def pinv(x, rcond=1e-15, hermitian=False, name=None):
    return _wrap(torch.linalg.pinv(x._t, rtol=rcond, hermitian=hermitian))


def svd(x, full_matrices=False, name=None):
    U, S, Vh = torch.linalg.svd(x._t, full_matrices=full_matrices)
    return _wrap(U), _wrap(S), _wrap(Vh)


def svdvals(x, name=None):
    return _wrap(torch.linalg.svdvals(x._t))


def qr(x, mode="reduced", name=None):
    Q, R = torch.linalg.qr(x._t, mode=mode)
    if mode == "r":
        return _wrap(R)
    return _wrap(Q), _wrap(R)


def lu(x, pivot=True, get_infos=False, name=None):
    LU, piv, info = torch.linalg.lu_factor_ex(x._t, pivot=pivot)
    out = (_wrap(LU), _wrap(piv.to(torch.int32)))
    return out + (_wrap(info.to(torch.int32)),) if get_infos else out


def eig(x, name=None):
    w_, v = torch.linalg.eig(x._t)
    return _wrap(w_), _wrap(v)


def eigvals(x, name=None):
    return _wrap(torch.linalg.eigvals(x._t))


def eigh(x, UPLO="L", name=None):
    w_, v = torch.linalg.eigh(x._t, UPLO=UPLO)
    return _wrap(w_), _wrap(v)


def eigvalsh(x, UPLO="L", name=None):
    return _wrap(torch.linalg.eigvalsh(x._t, UPLO=UPLO))


def solve(x, y, left=True, name=None):
    return _wrap(torch.linalg.solve(x._t, y._t, left=left))


def lstsq(x, y, rcond=None, driver=None, name=None):
    r = torch.linalg.lstsq(x._t, y._t, rcond=rcond, driver=driver)
    return _wrap(r.solution), _wrap(r.residuals), _wrap(r.rank), _wrap(r.singular_values)


def triangular_solve(x, y, upper=True, transpose=False, unitriangular=False, name=None):
    a = x._t.transpose(-1, -2) if transpose else x._t
    return _wrap(torch.linalg.solve_triangular(a, y._t, upper=upper != transpose, unitriangular=unitriangular))


def matrix_rank(x, tol=None, hermitian=False, atol=None, rtol=None, name=None):
    if tol is not None:
        atol = tol
    return _wrap(torch.linalg.matrix_rank(x._t, atol=atol, rtol=rtol, hermitian=hermitian))


def cond(x, p=None, name=None):
    return _wrap(torch.linalg.cond(x._t, p))


def cov(x, rowvar=True, ddof=True, fweights=None, aweights=None, name=None):
    t = x._t if rowvar else x._t.t()
    return _wrap(torch.cov(t, correction=int(ddof), fweights=None if fweights is None else fweights._t,
                           aweights=None if aweights is None else aweights._t))


def corrcoef(x, rowvar=True, name=None):
    return _wrap(torch.corrcoef(x._t if rowvar else x._t.t()))


def bincount(x, weights=None, minlength=0, name=None):
    return _wrap(torch.bincount(x._t, None if weights is None else weights._t, minlength))


def histogram(input, bins=100, min=0, max=0, weight=None, density=False, name=None):
    t = input._t.float()
    lo, hi = (float(min), float(max))
    if lo == 0 and hi == 0:
        lo, hi = t.min().item(), t.max().item()
    h = torch.histc(t, bins, lo, hi)
    return _wrap(h.to(torch.int64) if weight is None and not density else h)


def householder_product(x, tau, name=None):
    return _wrap(torch.linalg.householder_product(x._t, tau._t))


def matrix_exp(x, name=None):
    return _wrap(torch.linalg.matrix_exp(x._t))


def ormqr(x, tau, y, left=True, transpose=False, name=None):
    return _wrap(torch.ormqr(x._t, tau._t, y._t, left=left, transpose=transpose))


def lu_unpack(x, y, unpack_ludata=True, unpack_pivots=True, name=None):
    P, L, U = torch.lu_unpack(x._t, y._t.to(torch.int32), unpack_ludata, unpack_pivots)
    return _wrap(P), _wrap(L), _wrap(U)


def cdist(x, y, p=2.0, compute_mode="use_mm_for_euclid_dist_if_necessary", name=None):
    return _wrap(torch.cdist(x._t, y._t, p, compute_mode=compute_mode))


def transpose_last(x):
    return _wrap(ut(x).transpose(-1, -2))


__all__ = [_n for _n, _v in list(globals().items())
           if not _n.startswith("_") and callable(_v) and getattr(_v, "__module__", None) == __name__]
