"""paddle.sparse (COO/CSR) on torch sparse tensors (reference: python/paddle/sparse/)."""
from __future__ import annotations

import torch

from ..framework.tensor import Tensor

_w = Tensor._wrap


def sparse_coo_tensor(indices, values, shape=None, dtype=None, place=None, stop_gradient=True):
    i = indices._t if isinstance(indices, Tensor) else torch.as_tensor(indices)
    v = values._t if isinstance(values, Tensor) else torch.as_tensor(values)
    t = torch.sparse_coo_tensor(i, v, size=shape).coalesce()
    return _w(t)


def sparse_csr_tensor(crows, cols, values, shape, dtype=None, place=None, stop_gradient=True):
    c = crows._t if isinstance(crows, Tensor) else torch.as_tensor(crows)
    co = cols._t if isinstance(cols, Tensor) else torch.as_tensor(cols)
    v = values._t if isinstance(values, Tensor) else torch.as_tensor(values)
    return _w(torch.sparse_csr_tensor(c, co, v, size=shape))


def matmul(x, y, name=None):
    return _w(torch.sparse.mm(x._t, y._t) if x._t.is_sparse else torch.matmul(x._t, y._t))


def add(x, y, name=None):
    return _w(x._t + y._t)


def multiply(x, y, name=None):
    return _w(x._t * y._t)


def to_dense(x):
    return _w(x._t.to_dense())


def relu(x, name=None):
    t = x._t.coalesce()
    return _w(torch.sparse_coo_tensor(t.indices(), torch.relu(t.values()), t.shape))


def is_same_shape(x, y):
    return list(x.shape) == list(y.shape)


class nn:
    class ReLU:
        def __call__(self, x):
            return relu(x)
