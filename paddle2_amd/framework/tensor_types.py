"""Non-dense tensor types (reference: paddle/phi/core/selected_rows.h + selected_rows_impl.cc,
paddle/phi/core/tensor_array.h, paddle/phi/core/string_tensor.h, paddle/phi/kernels/strings/).

* ``SelectedRows`` — a row-sparse slice of a [height, ...] tensor: ``rows`` (int64 ids, may repeat) and
  ``value`` ([len(rows), ...]).  It is the gradient type of ``nn.Embedding(sparse=True)``; the optimizers update
  only the touched rows from it (SGD: one index_add; Adam ``lazy_mode``: moments of those rows only).
* ``TensorArray`` — the dense-tensor array behind ``paddle.tensor.create_array`` / ``array_write`` /
  ``array_read`` / ``array_length`` and ``tensor_array_to_tensor`` (a Python list of Tensors, in both modes: a
  recorded static program sees the writes as ordinary ops on the elements).
* ``StringTensor`` — an N-d array of UTF-8 strings with the phi string kernels (empty / copy / lower / upper,
  ASCII-only or full Unicode case mapping).
"""
from __future__ import annotations

import numpy as np
import torch


# ================================================================================================ SelectedRows
class SelectedRows:
    def __init__(self, rows=None, height=0, value=None):
        if rows is None:
            rows = torch.zeros(0, dtype=torch.int64)
        self._rows = torch.as_tensor(rows, dtype=torch.int64) if not isinstance(rows, torch.Tensor) else rows.long()
        self._height = int(height)
        self._value = _raw(value) if value is not None else None

    # ---------------------------------------------------------------- reference accessors
    def rows(self):
        return self._rows.tolist()

    def set_rows(self, rows):
        self._rows = torch.as_tensor(rows, dtype=torch.int64)

    def height(self):
        return self._height

    def set_height(self, h):
        self._height = int(h)

    def get_tensor(self):
        from .tensor import Tensor

        return Tensor._wrap(self._value)

    value = get_tensor

    def numel(self):
        return 0 if self._value is None else self._value.numel()

    @property
    def shape(self):
        return [self._height] + ([] if self._value is None else list(self._value.shape[1:]))

    @property
    def dtype(self):
        return None if self._value is None else self._value.dtype

    def has_key(self, key):
        return bool((self._rows == int(key)).any())

    def index(self, key):
        hit = (self._rows == int(key)).nonzero()
        if hit.numel() == 0:
            raise KeyError(f"key {key} not found in SelectedRows")
        return int(hit[0, 0])

    # ---------------------------------------------------------------- conversions
    @classmethod
    def from_torch_sparse(cls, g):
        """torch sparse COO gradient ([height, ...] with sparse dim 1) -> SelectedRows (rows kept as given)."""
        g = g.coalesce() if not g.is_coalesced() else g
        return cls(g.indices()[0], g.shape[0], g.values())

    def merge_add(self):
        """Sum rows with the same id (reference MergeAdd): unique sorted rows."""
        if self._rows.numel() == 0:
            return SelectedRows(self._rows, self._height, self._value)
        uniq, inv = torch.unique(self._rows.to(self._value.device), sorted=True, return_inverse=True)
        out = torch.zeros((uniq.numel(),) + tuple(self._value.shape[1:]), dtype=self._value.dtype,
                          device=self._value.device)
        out.index_add_(0, inv, self._value)
        return SelectedRows(uniq, self._height, out)

    def to_dense(self):
        out = torch.zeros([self._height] + list(self._value.shape[1:]), dtype=self._value.dtype,
                          device=self._value.device)
        out.index_add_(0, self._rows.to(self._value.device), self._value)
        return out

    def to_torch_sparse(self):
        return torch.sparse_coo_tensor(self._rows.unsqueeze(0).to(self._value.device), self._value,
                                       tuple(self.shape))

    def __repr__(self):
        return f"SelectedRows(height={self._height}, rows={self._rows.numel()}, value_shape={self.shape[1:]})"


def _raw(x):
    return x._t if hasattr(x, "_t") else (x if isinstance(x, torch.Tensor) else torch.as_tensor(np.asarray(x)))


# ================================================================================================ TensorArray
class TensorArray(list):
    """A list of Tensors with the reference's array ops; ``dtype`` is the element dtype it was created for."""

    def __init__(self, dtype=None, items=()):
        super().__init__(items)
        self.dtype = dtype

    def length(self):
        return len(self)


def _index(i):
    if isinstance(i, int):
        return i
    t = _raw(i)
    if t.numel() != 1:
        raise ValueError(f"The shape of index 'i' should be [1] or [], but got {list(t.shape)}")
    return int(t.reshape(-1)[0])


def create_array(dtype, initialized_list=None):
    from .tensor import Tensor

    items = []
    if initialized_list is not None:
        if not isinstance(initialized_list, (list, tuple)):
            raise TypeError(f"Require type(initialized_list) should be list/tuple, but received "
                            f"{type(initialized_list)}")
        for v in initialized_list:
            if not isinstance(v, Tensor):
                raise TypeError(f"All values in `initialized_list` should be Variable or pir.Value, but received "
                                f"{type(v)}.")
        items = list(initialized_list)
    return TensorArray(dtype, items)


def array_write(x, i, array=None):
    from .tensor import Tensor

    if not isinstance(x, Tensor):
        raise TypeError("The input data 'x' in array_write must be a Tensor")
    i = _index(i)
    if array is None:
        array = create_array(x.dtype)
    if not isinstance(array, list):
        raise TypeError("The 'array' in array_write must be a list / TensorArray")
    if i > len(array):
        raise IndexError("The index 'i' should not be greater than the length of 'array'")
    if i < len(array):
        array[i] = x
    else:
        array.append(x)
    return array


def array_read(array, i):
    if not isinstance(array, list):
        raise TypeError("The 'array' in array_read must be a list / TensorArray")
    return array[_index(i)]


def array_length(array):
    if not isinstance(array, list):
        raise TypeError("array should be a tensor array (list)")
    return len(array)


def tensor_array_to_tensor(input, axis=1, use_stack=False, name=None):
    """Concatenate (or stack) the array's tensors along ``axis``; also returns each element's size on it."""
    from .tensor import Tensor

    ts = [_raw(t) for t in input]
    out = torch.stack(ts, axis) if use_stack else torch.cat(ts, axis)
    sizes = torch.tensor([1 if use_stack else t.shape[axis] for t in ts], dtype=torch.int32)
    return Tensor._wrap(out), Tensor._wrap(sizes)


# ================================================================================================ StringTensor
class StringTensor:
    """N-d array of Python (UTF-8) strings."""

    def __init__(self, data=None, shape=None, name=None):
        if data is None:
            arr = np.full(tuple(shape or ()), "", dtype=object)
        else:
            arr = np.array(data, dtype=object)
            if shape is not None:
                arr = arr.reshape(shape)
        self._a = arr
        self.name = name

    @property
    def shape(self):
        return list(self._a.shape)

    def numel(self):
        return int(self._a.size)

    def numpy(self):
        return self._a.copy()

    def tolist(self):
        return self._a.tolist()

    def __getitem__(self, idx):
        r = self._a[idx]
        return StringTensor(r) if isinstance(r, np.ndarray) else r

    def __len__(self):
        return len(self._a)

    def __eq__(self, other):
        o = other._a if isinstance(other, StringTensor) else np.array(other, dtype=object)
        return self._a.shape == o.shape and bool((self._a == o).all())

    def __repr__(self):
        return f"StringTensor(shape={self.shape}, {self._a.tolist()!r})"


def _case(x, fn, use_utf8_encoding):
    def one(s):
        if use_utf8_encoding:
            return fn(s)
        # ASCII-only mapping: non-ASCII code points pass through unchanged
        return "".join(fn(c) if c.isascii() else c for c in s)

    out = np.vectorize(one, otypes=[object])(x._a) if x._a.size else x._a.copy()
    return StringTensor(out)


def strings_empty(shape):
    return StringTensor(shape=shape)


def strings_empty_like(x):
    return StringTensor(shape=x.shape)


def strings_copy(x):
    return StringTensor(x._a.copy())


def strings_lower(x, use_utf8_encoding=True):
    return _case(x, str.lower, use_utf8_encoding)


def strings_upper(x, use_utf8_encoding=True):
    return _case(x, str.upper, use_utf8_encoding)
