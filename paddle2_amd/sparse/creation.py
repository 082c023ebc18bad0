"""Sparse tensor creation and the sparse methods of Tensor (reference: python/paddle/sparse/creation.py,
paddle/phi/core/sparse_coo_tensor.h, sparse_csr_tensor.h).

Storage: a paddle Tensor whose ``_t`` is a torch ``sparse_coo`` (hybrid: ``sparse_dim`` index dims + dense
value dims, e.g. point-cloud features ``[N, D, H, W, C]`` with indices ``[4, nnz]`` and values ``[nnz, C]``, the
reference's SparseCooTensor layout) or ``sparse_csr`` (2-D ``[M, N]`` or batched 3-D ``[B, M, N]``) tensor.
Autograd flows through the values.
"""
from __future__ import annotations

import warnings

import torch

from ..framework.tensor import Tensor

_w = Tensor._wrap
warnings.filterwarnings("ignore", message="Sparse CSR tensor support is in beta")


def _u(x):
    return x._t if isinstance(x, Tensor) else (x if isinstance(x, torch.Tensor) else torch.as_tensor(x))


def _dt(dtype):
    if dtype is None:
        return None
    if isinstance(dtype, torch.dtype):
        return dtype
    from ..framework.dtype import convert_dtype

    return convert_dtype(dtype)


def _dev(place):
    if place is None:
        from ..framework.place import current_torch_device

        return current_torch_device()
    from ..framework.place import _parse_device

    return _parse_device(place)


def _finish(t, stop_gradient):
    o = _w(t)
    if not stop_gradient and t.is_floating_point():
        o.stop_gradient = False
    return o


def sparse_coo_tensor(indices, values, shape=None, dtype=None, place=None, stop_gradient=True):
    """COO tensor from indices [sparse_dim, nnz] and values [nnz, *dense_dims] (creation.py:60).  ``shape``
    defaults to (max index + 1) per sparse dim + the values' dense dims.  The result is coalesced (sorted,
    duplicates summed) like the reference's."""
    i = _u(indices).to(torch.int64)
    v = _u(values)
    if dtype is not None:
        v = v.to(_dt(dtype))
    dev = _dev(place) if place is not None else v.device
    i, v = i.to(dev), v.to(dev)
    if i.dim() != 2:
        raise ValueError("sparse_coo_tensor: indices must be 2-D [sparse_dim, nnz]")
    if shape is None:
        shape = [int(m) + 1 for m in (i.amax(1).tolist() if i.shape[1] else [0] * i.shape[0])] + list(v.shape[1:])
    shape = [int(s) for s in shape]
    if len(shape) != i.shape[0] + v.dim() - 1:
        raise ValueError(f"sparse_coo_tensor: shape {shape} vs indices {list(i.shape)} / values {list(v.shape)}")
    t = torch.sparse_coo_tensor(i, v, size=shape).coalesce()
    return _finish(t, stop_gradient)


def sparse_csr_tensor(crows, cols, values, shape, dtype=None, place=None, stop_gradient=True):
    """CSR tensor: 2-D [M, N] (crows [M+1]) or batched 3-D [B, M, N] (crows [B*(M+1)], per-batch row pointers as in
    the reference, creation.py:178)."""
    c = _u(crows).to(torch.int64)
    co = _u(cols).to(torch.int64)
    v = _u(values)
    if dtype is not None:
        v = v.to(_dt(dtype))
    dev = _dev(place) if place is not None else v.device
    c, co, v = c.to(dev), co.to(dev), v.to(dev)
    shape = [int(s) for s in shape]
    if len(shape) == 3:
        B, M = shape[0], shape[1]
        c = c.reshape(B, M + 1)
        nnz_b = (c[:, -1]).tolist()
        if len(set(nnz_b)) != 1:
            # torch batched CSR needs equal nnz per batch: pad each batch's rows with explicit zeros
            return _finish(_csr_from_coo(_batched_csr_to_coo(c, co, v, shape)), stop_gradient)
        co = co.reshape(B, -1)
        v = v.reshape(B, -1)
    t = torch.sparse_csr_tensor(c, co, v, size=shape)
    return _finish(t, stop_gradient)


def _batched_csr_to_coo(c, co, v, shape):
    B, M, _ = shape
    counts = (c[:, 1:] - c[:, :-1]).reshape(-1)
    rows = torch.repeat_interleave(torch.arange(B * M, device=c.device), counts)
    idx = torch.stack([rows // M, rows % M, co])
    return torch.sparse_coo_tensor(idx, v, size=shape).coalesce()


def _csr_from_coo(t):
    if t.dim() == 2:
        return t.to_sparse_csr()
    # batched: torch requires equal nnz per batch -> materialise explicit zeros for the short batches
    t = t.coalesce()
    B = t.shape[0]
    idx, val = t.indices(), t.values()
    nnz_b = torch.bincount(idx[0], minlength=B)
    mx = int(nnz_b.max()) if B else 0
    if bool((nnz_b == mx).all()):
        return t.to_sparse_csr()
    d = t.to_dense()
    mask = torch.zeros(d.shape, dtype=torch.bool, device=d.device)
    mask[tuple(idx)] = True
    real = mask.clone()
    # add zero entries (first free columns) until every batch has mx entries
    for b in range(B):
        need = mx - int(nnz_b[b])
        if need:
            free = (~mask[b]).reshape(-1).nonzero()[:need, 0]
            mask[b].view(-1)[free] = True
    return _masked_dense_to_csr(d, mask, real)


# Batched CSR tensors whose batches hold different nnz are stored with explicit-zero padding entries (torch needs
# equal nnz per batch); such a tensor carries the per-stored-value "real entry" mask (attribute _p2_real) so
# pattern-defined ops (softmax, attention, masked_matmul) ignore the padding.
def real_entries(t):
    """Bool per stored value (CSR value order) of the entries that belong to the pattern, or None if all do."""
    return getattr(t, "_p2_real", None)


def _masked_dense_to_csr(d, mask, real=None):
    B, M, N = d.shape
    nz = mask.nonzero()
    vals = d[mask]
    cnt = mask.sum(-1)  # [B, M]
    crow = torch.zeros(B, M + 1, dtype=torch.int64, device=d.device)
    crow[:, 1:] = cnt.cumsum(-1)
    t = torch.sparse_csr_tensor(crow, nz[:, 2].reshape(B, -1), vals.reshape(B, -1), size=(B, M, N))
    if real is not None:
        t._p2_real = real[mask].reshape(B, -1)
    return t


# ------------------------------------------------------------------------------------- Tensor methods
def _is_coo(t):
    return t.layout == torch.sparse_coo


def _is_csr(t):
    return t.layout == torch.sparse_csr


def to_coo_torch(t):
    """torch COO (coalesced) view of a COO or CSR torch tensor."""
    if _is_coo(t):
        return t if t.is_coalesced() else t.coalesce()
    if _is_csr(t):
        if t.dim() == 2:
            return t.to_sparse_coo().coalesce()
        B, M, N = t.shape
        crow, col, val = t.crow_indices(), t.col_indices(), t.values()
        counts = (crow[:, 1:] - crow[:, :-1]).reshape(-1)
        rows = torch.repeat_interleave(torch.arange(B * M, device=val.device), counts)
        idx = torch.stack([rows // M, rows % M, col.reshape(-1)])
        return torch.sparse_coo_tensor(idx, val.reshape(-1), size=t.shape).coalesce()
    raise TypeError("not a sparse tensor")


def _to_dense(self):
    t = self._t
    if _is_coo(t) or _is_csr(t):
        return _w(t.to_dense())
    return self


def _to_sparse_coo(self, sparse_dim=None):
    t = self._t
    if _is_coo(t):
        return self
    if _is_csr(t):
        return _w(to_coo_torch(t))
    sd = t.dim() if sparse_dim is None else int(sparse_dim)
    return _w(t.to_sparse(sd).coalesce())


def _to_sparse_csr(self):
    t = self._t
    if _is_csr(t):
        return self
    if _is_coo(t):
        if t.dense_dim():
            raise ValueError("to_sparse_csr: COO tensors with dense value dims have no CSR form")
        return _w(_csr_from_coo(t))
    if t.dim() == 2:
        return _w(t.to_sparse_csr())
    return _w(_csr_from_coo(t.to_sparse().coalesce()))


def _indices(self):
    return _w(to_coo_torch(self._t).indices())


def _values(self):
    t = self._t
    return _w(t.values() if _is_csr(t) and t.dim() == 2 else
              (t.values().reshape(-1) if _is_csr(t) else to_coo_torch(t).values()))


def _crows(self):
    t = self._t
    if not _is_csr(t):
        raise TypeError("crows() needs a CSR tensor")
    return _w(t.crow_indices().reshape(-1))


def _cols(self):
    t = self._t
    if not _is_csr(t):
        raise TypeError("cols() needs a CSR tensor")
    return _w(t.col_indices().reshape(-1))


def _nnz(self):
    t = self._t
    if _is_csr(t):
        return int(t.values().numel())
    return int(to_coo_torch(t)._nnz())


def _coalesce(self):
    return _w(to_coo_torch(self._t))


for _name, _fn in {
    "to_dense": _to_dense, "to_sparse_coo": _to_sparse_coo, "to_sparse_csr": _to_sparse_csr,
    "indices": _indices, "values": _values, "crows": _crows, "cols": _cols, "nnz": _nnz,
    "coalesce": _coalesce,
    "is_sparse": lambda self: _is_coo(self._t) or _is_csr(self._t),
    "is_sparse_coo": lambda self: _is_coo(self._t),
    "is_sparse_csr": lambda self: _is_csr(self._t),
}.items():
    setattr(Tensor, _name, _fn)
Tensor.is_dense = lambda self: not (_is_coo(self._t) or _is_csr(self._t))
