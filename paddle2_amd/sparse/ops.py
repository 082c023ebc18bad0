"""paddle.sparse math: unary (zero-preserving, applied to the stored values), binary, matmul family,
reductions and shape ops on COO / CSR tensors (reference: python/paddle/sparse/unary.py, binary.py,
multiary.py; phi/kernels/sparse/).

Products with a sparse operand are written as gather / index_add over the nonzeros (no densification):
``matmul(sparse, dense)`` = SpMM, ``masked_matmul(dense, dense, mask)`` = SDDMM (only the mask's nonzeros
are computed), both on any device with autograd through the values.
"""
from __future__ import annotations

import math

import torch

from ..framework.tensor import Tensor
from .creation import _csr_from_coo, _dt, _is_coo, _is_csr, _u, real_entries, to_coo_torch

_w = Tensor._wrap


def _rebuild(t, vals):
    """Same sparsity pattern as torch sparse tensor ``t``, new values."""
    if _is_csr(t):
        return torch.sparse_csr_tensor(t.crow_indices(), t.col_indices(), vals.reshape(t.values().shape), size=t.shape)
    c = to_coo_torch(t)
    return torch.sparse_coo_tensor(c.indices(), vals, size=c.shape, is_coalesced=True)


def _vals(t):
    return t.values() if _is_csr(t) else to_coo_torch(t).values()


def _unary(fn):
    def op(x, name=None):
        t = _u(x)
        return _w(_rebuild(t, fn(_vals(t))))
    op.__doc__ = f"Elementwise {fn.__name__ if hasattr(fn, '__name__') else 'op'} on the stored values."
    return op


sin = _unary(torch.sin)
tan = _unary(torch.tan)
asin = _unary(torch.asin)
atan = _unary(torch.atan)
sinh = _unary(torch.sinh)
tanh = _unary(torch.tanh)
asinh = _unary(torch.asinh)
atanh = _unary(torch.atanh)
sqrt = _unary(torch.sqrt)
square = _unary(torch.square)
log1p = _unary(torch.log1p)
abs = _unary(torch.abs)  # noqa: A001
neg = _unary(torch.neg)
expm1 = _unary(torch.expm1)
deg2rad = _unary(torch.deg2rad)
rad2deg = _unary(torch.rad2deg)
isnan = _unary(torch.isnan)
relu = _unary(torch.relu)


def pow(x, factor, name=None):  # noqa: A001
    t = _u(x)
    return _w(_rebuild(t, _vals(t) ** factor))


def cast(x, index_dtype=None, value_dtype=None, name=None):
    t = _u(x)
    vd = _dt(value_dtype)
    idt = _dt(index_dtype)
    v = _vals(t) if vd is None else _vals(t).to(vd)
    if _is_csr(t):
        ci, co = t.crow_indices(), t.col_indices()
        if idt is not None:
            ci, co = ci.to(idt), co.to(idt)
        return _w(torch.sparse_csr_tensor(ci, co, v.reshape(t.values().shape), size=t.shape))
    c = to_coo_torch(t)
    # torch COO indices are int64; index_dtype is accepted (the reference's int32 option) and kept as int64
    return _w(torch.sparse_coo_tensor(c.indices(), v, size=c.shape, is_coalesced=True))


def coalesce(x, name=None):
    return _w(to_coo_torch(_u(x)))


def is_same_shape(x, y):
    return list(_u(x).shape) == list(_u(y).shape)


# ------------------------------------------------------------------------------------------ binary
def _same_layout(x, t):
    return _w(_csr_from_coo(t) if _is_csr(x) else t)


def add(x, y, name=None):
    a, b = _u(x), _u(y)
    if not (a.is_sparse or _is_csr(a)) or not (b.is_sparse or _is_csr(b)):
        return _w(a.to_dense() + b.to_dense() if (a.is_sparse or _is_csr(a)) else a + b.to_dense())
    return _same_layout(a, (to_coo_torch(a) + to_coo_torch(b)).coalesce())


def subtract(x, y, name=None):
    a, b = _u(x), _u(y)
    return _same_layout(a, (to_coo_torch(a) - to_coo_torch(b)).coalesce())


def multiply(x, y, name=None):
    a, b = _u(x), _u(y)
    if isinstance(y, (int, float)):
        return _w(_rebuild(a, _vals(a) * y))
    if not (b.is_sparse or _is_csr(b)):  # sparse * dense: result keeps x's pattern
        return mask_as(_w(a.to_dense() * b), x)
    return _same_layout(a, (to_coo_torch(a) * to_coo_torch(b)).coalesce())


def divide(x, y, name=None):
    """x / y on x's nonzeros (y sparse with the same pattern, a dense tensor, or a scalar)."""
    a = _u(x)
    if isinstance(y, (int, float)):
        return _w(_rebuild(a, _vals(a) / y))
    b = _u(y)
    ca = to_coo_torch(a)
    yv = b.to_dense()[tuple(ca.indices())] if (b.is_sparse or _is_csr(b)) else b[tuple(ca.indices())]
    return _w(_rebuild(a, ca.values() / yv))


# ------------------------------------------------------------------------------------------ products
def _coords(t):
    c = to_coo_torch(t)
    return c.indices(), c.values(), c


def matmul(x, y, name=None):
    """sparse @ dense -> dense (SpMM over the nonzeros, batched for 3-D); sparse @ sparse -> sparse; dense @
    sparse -> dense."""
    a, b = _u(x), _u(y)
    a_sp, b_sp = a.is_sparse or _is_csr(a), b.is_sparse or _is_csr(b)
    if a_sp and b_sp:
        ca, cb = to_coo_torch(a), to_coo_torch(b)
        if a.dim() == 2:
            out = torch.sparse.mm(ca, cb).coalesce()
        else:
            out = torch.stack([torch.sparse.mm(ca[i], cb[i]) for i in range(a.shape[0])]).coalesce()
        return _same_layout(a, out)
    if a_sp:
        idx, val, c = _coords(a)
        if a.dim() == 2:  # out[i] += v * y[j]
            out = torch.zeros(a.shape[0], b.shape[-1], dtype=torch.result_type(val, b), device=b.device)
            return _w(out.index_add(0, idx[0], val[:, None] * b[idx[1]]))
        B, M = a.shape[0], a.shape[1]
        out = torch.zeros(B * M, b.shape[-1], dtype=torch.result_type(val, b), device=b.device)
        rows = idx[0] * M + idx[1]
        return _w(out.index_add(0, rows, val[:, None] * b[idx[0], idx[2]]).reshape(B, M, -1))
    if b_sp:  # dense @ sparse = (sparse^T @ dense^T)^T
        bt = transpose(_w(b), [1, 0] if b.dim() == 2 else [0, 2, 1])
        at = a.transpose(-1, -2)
        return _w(matmul(bt, _w(at))._t.transpose(-1, -2))
    return _w(torch.matmul(a, b))


def masked_matmul(x, y, mask, name=None):
    """SDDMM: (x @ y) evaluated only at ``mask``'s nonzeros -> sparse with mask's pattern and layout."""
    a, b, m = _u(x), _u(y), _u(mask)
    idx, _, c = _coords(m)
    if m.dim() == 2:
        vals = (a[idx[0]] * b[:, idx[1]].t()).sum(-1)
    else:
        vals = (a[idx[0], idx[1]] * b[idx[0], :, idx[2]]).sum(-1)
    real = real_entries(m)
    if real is not None:  # padding entries of a batched CSR mask stay zero
        vals = vals * real.reshape(-1).to(vals.dtype)
    out = torch.sparse_coo_tensor(idx, vals, size=c.shape, is_coalesced=True)
    return _same_layout(m, out)


def mask_as(x, mask, name=None):
    """Dense x sampled at mask's nonzeros (reference sparse.mask_as)."""
    a, m = _u(x), _u(mask)
    idx, _, c = _coords(m)
    vals = a[tuple(idx)]
    return _same_layout(m, torch.sparse_coo_tensor(idx, vals, size=c.shape, is_coalesced=True))


def mv(x, vec, name=None):
    return _w(matmul(x, _w(_u(vec)[:, None]))._t[:, 0])


def addmm(input, x, y, beta=1.0, alpha=1.0, name=None):  # noqa: A002
    prod = matmul(x, y)._t
    inp = _u(input)
    if inp.is_sparse or _is_csr(inp):
        if prod.is_sparse or _is_csr(prod):
            return add(_w(_rebuild(inp, beta * _vals(inp))), _w(_rebuild(prod, alpha * _vals(prod))))
        inp = inp.to_dense()
    return _w(beta * inp + alpha * prod)


def pca_lowrank(x, q=None, center=True, niter=2, name=None):
    t = to_coo_torch(_u(x))
    U, S, V = torch.pca_lowrank(t, q=q, center=center, niter=niter)
    return _w(U), _w(S), _w(V)


# ------------------------------------------------------------------------------------------ reductions / shape
def sum(x, axis=None, dtype=None, keepdim=False, name=None):  # noqa: A001
    t = _u(x)
    c = to_coo_torch(t)
    dt = _dt(dtype)
    if axis is None:
        v = c.values().sum()
        v = v.to(dt) if dt is not None else v
        shape = [1] * t.dim() if keepdim else [1]
        idx = torch.zeros(len(shape), 1, dtype=torch.int64, device=v.device)
        return _w(torch.sparse_coo_tensor(idx, v.reshape(1), size=shape, is_coalesced=True))
    axes = [axis] if isinstance(axis, int) else list(axis)
    axes = sorted(a % t.dim() for a in axes)
    sd = c.sparse_dim()
    if any(a >= sd for a in axes):  # reducing a dense value dim: reduce the values
        dense_axes = [a - sd + 1 for a in axes if a >= sd]
        vals = c.values().sum(dense_axes, keepdim=keepdim)
        shp = [s for i, s in enumerate(t.shape) if i < sd] + list(vals.shape[1:])
        c = torch.sparse_coo_tensor(c.indices(), vals, size=shp, is_coalesced=True)
        axes = [a for a in axes if a < sd]
        if not axes:
            out = c
            return _same_layout(t, out.to(dt) if dt is not None else out)
    keep = [i for i in range(c.sparse_dim()) if i not in axes]
    idx = c.indices()
    if keepdim:
        new_idx = idx.clone()
        new_idx[axes] = 0
        shape = [1 if i in axes else s for i, s in enumerate(c.shape)]
    else:
        new_idx = idx[keep]
        shape = [s for i, s in enumerate(c.shape) if i not in axes]
    vals = c.values() if dt is None else c.values().to(dt)
    if new_idx.shape[0] == 0:  # every sparse dim reduced: one stored entry of shape [1, *dense]
        v = vals.sum(0, keepdim=True)
        i0 = torch.zeros(1, 1, dtype=torch.int64, device=idx.device)
        return _w(torch.sparse_coo_tensor(i0, v, size=[1] + shape, is_coalesced=True))
    out = torch.sparse_coo_tensor(new_idx, vals, size=shape).coalesce()
    return _same_layout(t, out) if len(shape) >= 2 or not _is_csr(t) else _w(out)


def transpose(x, perm, name=None):
    t = _u(x)
    c = to_coo_torch(t)
    sd = c.sparse_dim()
    perm = [p % t.dim() for p in perm]
    if any(p >= sd for p in perm[:sd]):
        raise ValueError("sparse transpose: sparse and dense dims cannot be exchanged")
    idx = c.indices()[perm[:sd]]
    shape = [c.shape[p] for p in perm]
    vals = c.values()
    if len(perm) > sd:
        vals = vals.permute([0] + [p - sd + 1 for p in perm[sd:]])
    out = torch.sparse_coo_tensor(idx, vals, size=shape).coalesce()
    return _same_layout(t, out)


def reshape(x, shape, name=None):
    """Reshape the sparse dims (dense value dims keep their shape): linearise indices, re-split."""
    t = _u(x)
    c = to_coo_torch(t)
    sd = c.sparse_dim()
    old = list(c.shape[:sd])
    dense = list(c.shape[sd:])
    shape = list(shape)
    total = math.prod(old)
    new_sp = shape[:len(shape) - len(dense)] if dense else shape
    if -1 in new_sp:
        k = new_sp.index(-1)
        new_sp[k] = total // max(1, math.prod(s for s in new_sp if s != -1))
    if math.prod(new_sp) != total:
        raise ValueError(f"sparse reshape: {old} -> {new_sp}")
    lin = torch.zeros(c.indices().shape[1], dtype=torch.int64, device=c.device)
    for d, s in enumerate(old):
        lin = lin * s + c.indices()[d]
    idx = []
    for s in reversed(new_sp):
        idx.append(lin % s)
        lin = lin // s
    idx = torch.stack(idx[::-1])
    out = torch.sparse_coo_tensor(idx, c.values(), size=new_sp + dense).coalesce()
    return _same_layout(t, out) if (not _is_csr(t) or len(new_sp) in (2, 3)) else _w(out)


def slice(x, axes, starts, ends, name=None):  # noqa: A001
    t = _u(x)
    c = to_coo_torch(t)
    idx, vals = c.indices(), c.values()
    shape = list(c.shape)
    keep = torch.ones(idx.shape[1], dtype=torch.bool, device=idx.device)
    idx = idx.clone()
    for a, s, e in zip(axes, starts, ends):
        a = a % t.dim()
        n = shape[a]
        s = max(0, s + n if s < 0 else s)
        e = min(n, e + n if e < 0 else e)
        keep &= (idx[a] >= s) & (idx[a] < e)
        idx[a] -= s
        shape[a] = max(0, e - s)
    out = torch.sparse_coo_tensor(idx[:, keep], vals[keep], size=shape).coalesce()
    return _same_layout(t, out)
