"""paddle.linalg namespace (reference: python/paddle/linalg.py)."""
from .tensor.linalg import (cholesky, cholesky_solve, cond, corrcoef, cov, det, eig, eigh, eigvals,  # noqa: F401
                            eigvalsh, householder_product, inv, inverse, lstsq, lu, lu_unpack, matrix_exp,
                            matrix_norm, matrix_power, matrix_rank, multi_dot, norm, ormqr, pinv, qr, slogdet, solve,
                            svd, svdvals, triangular_solve, vector_norm, cross, matmul, vecdot, cdist)
