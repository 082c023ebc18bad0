"""paddle.sparse — COO / CSR sparse tensors and their ops (reference: python/paddle/sparse/, 5.6 k LoC, and
paddle/phi/kernels/sparse/).  See creation.py (storage + Tensor methods), ops.py (math), nn/ (sparse
convolution via rulebook + grouped MFMA GEMM, pooling, activations, softmax, attention, batch norm)."""
from __future__ import annotations

from . import nn  # noqa: F401
from .creation import sparse_coo_tensor, sparse_csr_tensor  # noqa: F401
from .ops import (abs, add, addmm, asin, asinh, atan, atanh, cast, coalesce, deg2rad, divide, expm1,  # noqa: F401
                  is_same_shape, isnan, log1p, mask_as, masked_matmul, matmul, multiply, mv, neg, pca_lowrank,
                  pow, rad2deg, reshape, sin, sinh, slice, sqrt, square, subtract, sum, tan, tanh, transpose)

__all__ = ["sparse_coo_tensor", "sparse_csr_tensor", "sin", "tan", "asin", "atan", "sinh", "tanh", "asinh", "atanh",
           "sqrt", "square", "log1p", "abs", "pow", "pca_lowrank", "cast", "neg", "deg2rad", "rad2deg", "expm1", "mv",
           "matmul", "mask_as", "masked_matmul", "addmm", "add", "subtract", "transpose", "sum", "multiply", "divide",
           "coalesce", "is_same_shape", "reshape", "isnan", "slice"]


def to_dense(x):
    return x.to_dense()


def relu(x, name=None):
    return nn.functional.relu(x)
