"""Tensor-array ops (reference: python/paddle/tensor/array.py): create_array / array_write / array_read /
array_length, plus tensor_array_to_tensor.  The array is a ``TensorArray`` (framework/tensor_types.py)."""
from ..framework.tensor_types import (array_length, array_read, array_write, create_array,  # noqa: F401
                                      tensor_array_to_tensor)

__all__ = ["array_length", "array_read", "array_write", "create_array", "tensor_array_to_tensor"]
